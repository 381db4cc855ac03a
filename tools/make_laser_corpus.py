#!/usr/bin/env python3
"""Write tests/golden/laser/: LASER-shaped feasibility queries derived from the
reference's own runtime bytecode.

Source bytecode: the reference's runtime-bytecode fixtures (data), copied to
tests/golden/laser_bytecode.json (or read from a checkout with --ref):
tests/testdata/inputs/
  underflow.sol.o  = solidity_examples/token.sol (transfer renamed sendeth) — C2's contract
  overflow.sol.o, metacoin.sol.o — the same mapping/arithmetic shapes
  suicide.sol.o    = C1's contract (suicide.sol, kill(address))

Each contract runs a 2-3 transaction sequence under tests/laser_concolic.py
(symbolic calldata, caller, callvalue; a concrete path chosen by the listed
inputs); every JUMPI contributes both successor sets (LASER prunes each with
is_possible, svm.py:287-292).  The followed successor is SAT and its model is
verified here with the oracle; the other successor's status is unknown.
Output: one ``--solver-log``-format file per query (z3 Optimize.sexpr shape,
mythril/support/model.py:45-56), gzip-compressed, starting with
``; expect: sat|unknown``, plus
manifest.json (per query: contract, tx, pc, status, the SAT model's scalar
leaves).

    python tools/make_laser_corpus.py [--ref /root/reference] [--only contract/scenario --out DIR]
"""
import argparse
import gzip
import io
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mythril_amd.smt2 import to_smt2  # noqa: E402
from oracle.keccak import keccak256  # noqa: E402
from tests.laser_concolic import ACTORS, TxInput, abi_call, check_model, run_sequence  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "laser")


def sel(sig: str) -> int:
    return int.from_bytes(keccak256(sig.encode())[:4], "big")


A, C, S = ACTORS["ATTACKER"], ACTORS["CREATOR"], ACTORS["SOMEGUY"]

# contract -> list of (scenario name, [TxInput...])
SCENARIOS = {
    "underflow": [   # token.sol: sendeth(to, value) twice, then balanceOf
        ("t3_send_send_balance", [
            TxInput(abi_call(sel("sendeth(address,uint256)"), S, 5), sender=A),
            TxInput(abi_call(sel("sendeth(address,uint256)"), A, 2), sender=S),
            TxInput(abi_call(sel("balanceOf(address)"), A), sender=C)]),
        ("t2_underflowing_send", [
            TxInput(abi_call(sel("sendeth(address,uint256)"), S, 1 << 200), sender=A),
            TxInput(abi_call(sel("totalSupply()")), sender=S)]),
        ("t2_short_calldata", [
            TxInput(sel("sendeth(address,uint256)").to_bytes(4, "big") + b"\x00" * 20, sender=A),
            TxInput(abi_call(sel("balanceOf(address)"), S), sender=A, value=0)]),
    ],
    "overflow": [
        ("t3_send_send_balance", [
            TxInput(abi_call(sel("sendeth(address,uint256)"), A, 7), sender=C),
            TxInput(abi_call(sel("sendeth(address,uint256)"), C, 3), sender=A),
            TxInput(abi_call(sel("balanceOf(address)"), C), sender=S)]),
    ],
    "metacoin": [
        ("t3_sendtoken", [
            TxInput(abi_call(sel("sendToken(address,uint256)"), S, 0), sender=A),
            TxInput(abi_call(sel("sendToken(address,uint256)"), A, 10), sender=S),
            TxInput(abi_call(sel("balances(address)"), A), sender=C)]),
    ],
    "suicide": [   # config C1's contract: kill(addr) after a failed and a bad-selector call
        ("t2_kill", [
            TxInput(abi_call(0xDEADBEEF), sender=S),
            TxInput(abi_call(sel("kill(address)"), A), sender=A)]),
        ("t2_value_reverts", [
            TxInput(abi_call(sel("kill(address)"), C), sender=C, value=5),
            TxInput(abi_call(sel("kill(address)"), S), sender=A)]),
    ],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default=None, help="read the .sol.o files from a reference checkout "
                    "instead of tests/golden/laser_bytecode.json")
    ap.add_argument("--out", default=OUT)
    ap.add_argument("--only", default=None, help="contract/scenario to (re)generate")
    a = ap.parse_args()
    write(a.out, a.ref, a.only)


def load_code(contract: str, ref=None) -> bytes:
    if ref:
        path = os.path.join(ref, "tests", "testdata", "inputs", f"{contract}.sol.o")
        return bytes.fromhex(open(path).read().strip())
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "laser_bytecode.json")))
    return bytes.fromhex(d["bytecode"][contract])


def write(out_dir: str, ref=None, only=None):
    os.makedirs(out_dir, exist_ok=True)
    if only is None:
        for f in os.listdir(out_dir):
            os.unlink(os.path.join(out_dir, f))
    manifest = []
    for contract, scenarios in SCENARIOS.items():
        code = load_code(contract, ref)
        for name, txs in scenarios:
            if only is not None and only != f"{contract}/{name}":
                continue
            m, run = run_sequence(code, txs, balances={x: 10 ** 18 for x in ACTORS.values()})
            for qi, q in enumerate(run.queries):
                if q.sat:
                    assert check_model(q.constraints, run.model), (contract, name, qi)
                fn = f"{contract}_{name}_q{qi:02d}_{'sat' if q.sat else 'unknown'}.smt2.gz"
                with io.TextIOWrapper(gzip.GzipFile(os.path.join(out_dir, fn), "wb", 9, mtime=0)) as fh:
                    fh.write(f"; expect: {'sat' if q.sat else 'unknown'}\n")
                    fh.write(f"; source: reference tests/testdata/inputs/{contract}.sol.o, tx {q.tx}, "
                             f"JUMPI at pc {q.pc}, {'followed' if q.taken else 'other'} successor\n")
                    fh.write(to_smt2(q.constraints))
                scalars = {k: hex(v) for k, v in run.model.items() if isinstance(v, int)}
                manifest.append({"file": fn, "contract": contract, "scenario": name, "tx": q.tx, "pc": q.pc,
                                 "status": "sat" if q.sat else "unknown", "conjuncts": len(q.constraints),
                                 "model_scalars": scalars if q.sat else None})
            print(f"{contract}/{name}: {len(run.queries)} queries, tx results {run.halts}")
    if only is None:
        json.dump(manifest, open(os.path.join(out_dir, "manifest.json"), "w"), indent=1)
    print(f"{len(manifest)} queries -> {out_dir}")
    return manifest


if __name__ == "__main__":
    main()
