"""ORACLE (test infrastructure only): run a VMTests fixture through MiniEVM.

Mirrors the assertion of ``tests/laser/evm_testsuite/evm_test.py:165-189``:
only the post-storage keys the fixture lists are compared (a Bool stored value
counts as 1/0, ``:181-183``).
"""
from __future__ import annotations

from mythril_amd.ir import Ctx, BOOL
from .evm import MiniEVM, Unsupported, EvmHalt


def h(x: str) -> int:
    return int(x, 16) if x not in ("", "0x") else 0


def env_of(case: dict) -> dict:
    e = case["env"]
    data = bytes.fromhex(case["data"][2:])
    return {"address": h(case["address"]), "origin": h(case["origin"]),
            "caller": h(case["caller"]), "value": h(case["value"]), "data": data,
            "gasPrice": h(case["gasPrice"]), "coinbase": h(e["currentCoinbase"]),
            "timestamp": h(e["currentTimestamp"]), "number": h(e["currentNumber"]),
            "difficulty": h(e["currentDifficulty"]), "gaslimit": h(e["currentGasLimit"])}


def run_case(case: dict, ctx: Ctx = None):
    """Returns (status, evm, checks) with checks = [(slot, term, expected)].

    status: 'ok' | 'unsupported' | 'halt'
    """
    ctx = ctx or Ctx()
    evm = MiniEVM(ctx, env_of(case))
    for k, v in case["pre_storage"].items():
        evm.storage[h(k)] = ctx.const(h(v), 256)
    try:
        evm.run(bytes.fromhex(case["code"][2:]))
    except Unsupported:
        return "unsupported", evm, []
    except EvmHalt:
        return "halt", evm, []
    checks = []
    for k, v in case["post_storage"].items():
        term = evm.storage.get(h(k), ctx.const(0, 256))
        checks.append((h(k), term, h(v)))
    return "ok", evm, checks


def concrete(evm: MiniEVM, term) -> int:
    v = evm.v(term)
    return int(v) if term.width != BOOL else (1 if v else 0)
