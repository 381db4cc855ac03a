#!/usr/bin/env python3
"""Write tests/golden/laser/: LASER-shaped feasibility queries derived from the
reference's own runtime bytecode.

Source bytecode: the reference's bytecode fixtures (data), copied to
tests/golden/laser_bytecode.json (or read from a checkout with --ref):
tests/testdata/inputs/
  underflow.sol.o  = solidity_examples/token.sol (transfer renamed sendeth) — C2's contract
  overflow.sol.o, metacoin.sol.o — the same mapping/arithmetic shapes
  suicide.sol.o    = C1's contract (suicide.sol, kill(address))
  flag_array.sol.o — CREATION code; extractMoney's EtherThief query, pinned by the
                     reference's expected calldata (tests/integration_tests/analysis_tests.py:9-19)
  origin.sol.o, calls.sol.o, kinds_of_calls.sol.o, returnvalue.sol.o, ether_send.sol.o
                   — ORIGIN, the four CALL kinds to symbolic callees ({tx}_retval_{pc}),
                     BALANCE, the call-site module queries
  exceptions_0.8.0.sol.o — creation code, Panic paths, the Power UF (EXP)
  environments.sol.o — batchTransfer(address[],uint256): the BECToken shape of C3
tests/laser/evm_testsuite/VMTests/vmIOandFlowOperations/DynamicJumpJD_DependsOnJumps{0,1}.json
                   — NUMBER in a JUMPI condition (block_number)

Each contract runs a 1-3 transaction sequence under tests/laser_concolic.py
(symbolic calldata, caller, callvalue; a concrete path chosen by the listed
inputs); every JUMPI contributes both successor sets (LASER prunes each with
is_possible, svm.py:287-292).  The followed successor is SAT and its model is
verified here with the oracle; the other successor's status is unknown.  The
detection modules' own get_model queries along the path are recorded too
(``kind``: EtherThief, StateChangeAfterCall/*, IntegerArithmetics/*), SAT when
the concrete model satisfies them, else unknown.
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
from tests.laser_concolic import ACTORS, CONTRACT, TxInput, abi_call, asm, check_model, run_sequence  # noqa: E402

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
    # creation code: tx 1 is CREATOR's creation with 0.1 ether (the constructor's
    # require), tx 2 the reference's EtherThief test case (analysis_tests.py:9-19)
    "flag_array": [
        ("t2_extract_money", [
            TxInput(b"", sender=C, value=10 ** 17, creation=True),
            TxInput(abi_call(sel("extractMoney(uint256)"), 1234), sender=A)]),
        ("t2_unflagged_index", [
            TxInput(b"", sender=C, value=10 ** 17, creation=True),
            TxInput(abi_call(sel("extractMoney(uint256)"), 77), sender=A)]),
    ],
    "origin": [   # the runtime code's storage is symbolic: the model's owner (slot 0) decides the ORIGIN check
        ("t2_transfer_ownership", [
            TxInput(abi_call(sel("transferOwnership(address)"), S), sender=A),
            TxInput(abi_call(sel("owner()")), sender=C)], {"storage": {0: A}}),
        ("t1_origin_check_fails", [
            TxInput(abi_call(sel("transferOwnership(address)"), S), sender=A)]),
    ],
    "calls": [
        ("t3_stored_and_user_address", [
            TxInput(abi_call(sel("setstoredaddress(address)"), A), sender=A),
            TxInput(abi_call(sel("callstoredaddress()")), sender=A),
            TxInput(abi_call(sel("calluseraddress(address)"), S), sender=S)]),
        ("t2_fixed_address", [
            TxInput(abi_call(sel("thisisfine()")), sender=A),
            TxInput(abi_call(sel("reentrancy()")), sender=C, retvals={-1: 0})]),
    ],
    "kinds_of_calls": [
        ("t3_call_kinds", [
            TxInput(abi_call(sel("callSetN(address,uint256)"), A, 5), sender=A),
            TxInput(abi_call(sel("callcodeSetN(address,uint256)"), S, 1), sender=S),
            TxInput(abi_call(sel("delegatecallSetN(address,uint256)"), A, 2), sender=A)]),
    ],
    "returnvalue": [
        ("t2_checked_unchecked", [
            TxInput(abi_call(sel("callnotchecked()")), sender=A, retvals={-1: 0}),
            TxInput(abi_call(sel("callchecked()")), sender=S)]),
        ("t1_failed_checked_call", [
            TxInput(abi_call(sel("callchecked()")), sender=A, retvals={-1: 0})]),
    ],
    "ether_send": [
        ("t3_crowdfund_invest_withdraw", [
            TxInput(abi_call(sel("crowdfunding()")), sender=A),
            TxInput(abi_call(sel("invest()")), sender=S, value=2 * 10 ** 18),
            TxInput(abi_call(sel("withdrawfunds()")), sender=A)],
         {"balances": 10 ** 20, "storage": {2: 10 ** 18, 3: 10 * 10 ** 18}}),   # INVEST_MIN, INVEST_MAX
    ],
    # analysis_tests.py:21-31: -t 1 -m Exceptions reports two issues, assert1() and
    # fail() (val is 0 after the creation); change_val() reaches none
    "exceptions_0.8.0": [
        ("t2_assert_fails", [
            TxInput(b"", sender=C, creation=True),
            TxInput(abi_call(sel("assert1()")), sender=A)]),
        ("t2_fail", [
            TxInput(b"", sender=C, creation=True),
            TxInput(abi_call(sel("fail()")), sender=S)]),
        ("t2_change_val", [
            TxInput(b"", sender=C, creation=True),
            TxInput(abi_call(sel("change_val()")), sender=A)]),
        ("t3_change_then_fail", [
            TxInput(b"", sender=C, creation=True),
            TxInput(abi_call(sel("change_val()")), sender=A),
            TxInput(abi_call(sel("fail()")), sender=S)]),
    ],
    # BECToken's batchTransfer (C3's shape) in the reference's own bytecode: the
    # receivers array is ABI-encoded (offset 0x40, length, addresses)
    "environments": [
        ("t1_batch_transfer", [
            TxInput(abi_call(sel("batchTransfer(address[],uint256)"), 0x40, 5, 2, A, S), sender=A)]),
        ("t1_batch_transfer_overflow", [
            TxInput(abi_call(sel("batchTransfer(address[],uint256)"), 0x40, 1 << 255, 2, A, S), sender=S)]),
    ],
    # Solidity 0.5 asserts end in INVALID: the Exceptions module's INVALID pre hook
    # (exceptions.py:62-84); requireisfine / thisisfine / thisisalsofind reach none
    "exceptions": [
        ("t1_assert1", [TxInput(abi_call(sel("assert1()")), sender=A)]),
        ("t1_assert3_23", [TxInput(abi_call(sel("assert3(uint256)"), 23), sender=S)]),
        ("t1_division_by_zero", [TxInput(abi_call(sel("divisionby0(uint256)"), 0), sender=A)]),
        ("t1_array_out_of_bounds", [TxInput(abi_call(sel("arrayaccess(uint256)"), 8), sender=C)]),
        ("t3_fine_paths", [
            TxInput(abi_call(sel("thisisfine(uint256)"), 5), sender=A),
            TxInput(abi_call(sel("thisisalsofind(uint256)"), 3), sender=S),
            TxInput(abi_call(sel("requireisfine(uint256)"), 22), sender=A)]),
    ],
    # msg.sender.transfer(1 ether): a CALL with value to the (symbolic) caller,
    # the contract's own balance symbolic in the starting world state
    "multi_contracts": [
        ("t2_transfer_twice", [
            TxInput(abi_call(sel("transfer()")), sender=A),
            TxInput(abi_call(sel("transfer()")), sender=S)], {"contract_balance": 5 * 10 ** 18}),
    ],
    "nonascii": [
        ("t2_render", [
            TxInput(abi_call(sel("renderNonAscii()")), sender=A),
            TxInput(abi_call(0x12345678), sender=S)]),
    ],
    # the runtime code of tests/testdata/input_contracts/safe_funcs.sol (0.8:
    # assert -> Panic(0x01) REVERT, the Exceptions REVERT pre hook), symbolic storage
    "safe_funcs": [
        ("t2_change_then_fail", [
            TxInput(abi_call(sel("change_val()")), sender=A),
            TxInput(abi_call(sel("fail()")), sender=S)]),
        ("t1_fail_holds", [TxInput(abi_call(sel("fail()")), sender=A)], {"storage": {0: 2}}),
        ("t1_assert1", [TxInput(abi_call(sel("assert1()")), sender=C)]),
    ],
    # creation code with a constructor argument (CODESIZE / CODECOPY past the
    # code read the creation's symbolic calldata, instructions.py:977-993,
    # 1065-1130) that becomes an immutable patched into the runtime code;
    # analysis_tests.py:32-41: -t 1 -m AccidentallyKillable reports one issue
    "symbolic_exec_bytecode": [
        ("t2_commence_killing", [
            TxInput((5).to_bytes(32, "big").ljust(0x200, b"\0"), sender=C, creation=True),
            TxInput(abi_call(sel("commencekilling()")), sender=A)]),
        ("t2_get_bytes", [
            TxInput((5).to_bytes(32, "big").ljust(0x200, b"\0"), sender=C, creation=True),
            TxInput(abi_call(sel("getBytes(bytes)"), 0x20, 3, 0xABCDEF << 232), sender=S)]),
        ("t2_get_bytes_too_long", [
            TxInput((1).to_bytes(32, "big").ljust(0x200, b"\0"), sender=C, creation=True),
            TxInput(abi_call(sel("getBytes(bytes)"), 0x20, 3, 0xABCDEF << 232), sender=A)]),
    ],
    # SYNTHETIC (builder-written; no reference fixture reaches BLOCKHASH): the
    # lottery shape `blockhash(block.number - 1) % 2 == 0` plus a timestamp
    # check, for PredictableVars' BLOCKHASH and JUMPI queries
    # (dependence_on_predictable_vars.py:68-82,142-159)
    "synthetic:predictable": [
        ("t1_blockhash_lottery", [TxInput(b"", sender=A, env={"blockhash_block_block_number - 1": 0x1234,
                                                               "timestamp": 0x60000001})]),
        ("t1_blockhash_odd", [TxInput(b"", sender=S, env={"blockhash_block_block_number - 1": 0x1235})]),
    ],
    "vm:vmIOandFlowOperations/DynamicJumpJD_DependsOnJumps0": [
        ("t1_number_branch", [TxInput(b"", sender=A, env={"block_number": 1})]),
        ("t1_number_zero", [TxInput(b"", sender=A, env={"block_number": 0})]),
    ],
    "vm:vmIOandFlowOperations/DynamicJumpJD_DependsOnJumps1": [
        ("t1_number_branch", [TxInput(b"", sender=A, env={"block_number": 5})]),
    ],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default=None, help="read the .sol.o files from a reference checkout "
                    "instead of tests/golden/laser_bytecode.json")
    ap.add_argument("--out", default=OUT)
    ap.add_argument("--only", default=None, help="contract/scenario to (re)generate")
    ap.add_argument("--import-bytecode", action="store_true", help="copy the fixtures from --ref into "
                    "tests/golden/laser_bytecode.json first")
    a = ap.parse_args()
    if a.import_bytecode:
        import_bytecode(a.ref)
    write(a.out, a.ref, a.only)


def synthetic_code(name: str) -> bytes:
    """SYNTHETIC contracts (builder-written, tests/laser_concolic.py asm)."""
    assert name == "predictable"
    NUMBER, BLOCKHASH, TIMESTAMP, SUB, MOD, ISZERO, GT, JUMPI, STOP = 0x43, 0x40, 0x42, 0x03, 0x06, 0x15, 0x11, 0x57, 0x00
    CALLVALUE, SSTORE, SWAP1 = 0x34, 0x55, 0x90
    return asm([
        ("push", 1, 1), NUMBER, SUB, BLOCKHASH,                  # blockhash(block.number - 1)
        ("push", 1, 2), SWAP1, MOD, ISZERO, ("ref", "win"), JUMPI, STOP,   # ... % 2 == 0
        ("label", "win"), ("push", 4, 0x60000000), TIMESTAMP, GT, ("ref", "late"), JUMPI, STOP,
        ("label", "late"), CALLVALUE, ("push", 1, 0), SSTORE, STOP,
    ])


def load_code(contract: str, ref=None) -> bytes:
    """The bytecode of a fixture: ``name`` is tests/testdata/inputs/name.sol.o,
    ``vm:category/test`` the ``exec.code`` of a VMTests json, ``synthetic:x``
    a builder-written contract (synthetic_code)."""
    if contract.startswith("synthetic:"):
        return synthetic_code(contract.split(":", 1)[1])
    if ref:
        if contract.startswith("vm:"):
            path = os.path.join(ref, "tests", "laser", "evm_testsuite", "VMTests", contract[3:] + ".json")
            d = json.load(open(path))
            return bytes.fromhex(next(iter(d.values()))["exec"]["code"][2:])
        path = os.path.join(ref, "tests", "testdata", "inputs", f"{contract}.sol.o")
        return bytes.fromhex(open(path).read().strip())
    d = json.load(open(os.path.join(ROOT, "tests", "golden", "laser_bytecode.json")))
    return bytes.fromhex(d["bytecode"][contract])


def import_bytecode(ref: str) -> None:
    """Copy every fixture SCENARIOS names from a reference checkout into
    tests/golden/laser_bytecode.json (data: hex strings)."""
    path = os.path.join(ROOT, "tests", "golden", "laser_bytecode.json")
    d = json.load(open(path))
    for contract in SCENARIOS:
        if not contract.startswith("synthetic:"):
            d["bytecode"][contract] = load_code(contract, ref).hex()
    d["source"] = ("runtime / creation bytecode of /root/reference/tests/testdata/inputs/*.sol.o and exec.code "
                   "of tests/laser/evm_testsuite/VMTests/*/*.json (reference test data)")
    json.dump(d, open(path, "w"), indent=1)


def scenario_balances(opts) -> dict:
    """The starting balances of the model: every actor's, and the contract's own
    when the scenario names one (its balance is symbolic in LASER's world state)."""
    bal = opts.get("balances", 10 ** 18)
    out = {x: bal for x in ACTORS.values()}
    if "contract_balance" in opts:
        out[CONTRACT] = opts["contract_balance"]
    return out


def write(out_dir: str, ref=None, only=None):
    os.makedirs(out_dir, exist_ok=True)
    if only is None:
        for f in os.listdir(out_dir):
            os.unlink(os.path.join(out_dir, f))
    manifest = []
    for contract, scenarios in SCENARIOS.items():
        code = load_code(contract, ref)
        for name, txs, *opt in scenarios:
            if only is not None and only != f"{contract}/{name}":
                continue
            opts = opt[0] if opt else {}
            m, run = run_sequence(code, txs, storage=opts.get("storage"), balances=scenario_balances(opts))
            for qi, q in enumerate(run.queries):
                if q.sat:
                    assert check_model(q.constraints, run.model), (contract, name, qi)
                tag = contract.replace("vm:", "vm_").replace("synthetic:", "synthetic_").replace("/", "_")
                kt = "" if q.kind == "jumpi" else q.kind.replace("/", "-") + "_"
                fn = f"{tag}_{name}_q{qi:02d}_{kt}{'sat' if q.sat else 'unknown'}.smt2.gz"
                with io.TextIOWrapper(gzip.GzipFile(os.path.join(out_dir, fn), "wb", 9, mtime=0)) as fh:
                    fh.write(f"; expect: {'sat' if q.sat else 'unknown'}\n")
                    src = (f"tests/laser/evm_testsuite/VMTests/{contract[3:]}.json" if contract.startswith("vm:")
                           else "SYNTHETIC (builder-written) " + contract if contract.startswith("synthetic:")
                           else f"tests/testdata/inputs/{contract}.sol.o")
                    where = (f"JUMPI at pc {q.pc}, {'followed' if q.taken else 'other'} successor" if q.kind == "jumpi"
                             else f"{q.kind} get_model at pc {q.pc}")
                    fh.write(f"; source: reference {src}, tx {q.tx}, {where}\n")
                    fh.write(to_smt2(q.constraints))
                scalars = {k: hex(v) for k, v in run.model.items() if isinstance(v, int)}
                manifest.append({"file": fn, "contract": contract, "scenario": name, "tx": q.tx, "pc": q.pc,
                                 "kind": q.kind, "status": "sat" if q.sat else "unknown",
                                 "tuple": q.tuple_form,
                                 "conjuncts": len(q.constraints),
                                 "model_scalars": scalars if q.sat else None})
            kinds = {}
            for q in run.queries:
                kinds[q.kind] = kinds.get(q.kind, 0) + 1
            print(f"{contract}/{name}: {len(run.queries)} queries {kinds}, tx results {run.halts}")
    if only is None:
        json.dump(manifest, open(os.path.join(out_dir, "manifest.json"), "w"), indent=1)
    print(f"{len(manifest)} queries -> {out_dir}")
    return manifest


if __name__ == "__main__":
    main()
