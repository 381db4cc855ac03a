#!/usr/bin/env python3
"""Write tests/golden/solver_log/*.smt2: feasibility queries in the
``--solver-log`` format (z3 ``Optimize.sexpr()``, mythril/support/model.py:45-56)
with the shapes LASER builds for the BASELINE.json contracts — synthetic
(no z3/solc here to dump real runs), restated from the reference:

* c2_token_*: solidity_examples/token.sol ``transfer`` (line 12-15): dispatcher
  selector JUMPI, calldatasize bound, ``balances[msg.sender]`` as a Storage read
  at keccak256_512(sender . slot 0), SWC-101 ``Not(BVSubNoUnderflow)``
  (mythril/analysis/module/modules/integer.py:141-160);
* c3_bec_*: solidity_examples/BECToken.sol ``batchTransfer`` (line 254-258):
  dynamic-array length read at a symbolic calldata offset, ``cnt > 0 && cnt <= 20``,
  ``Not(BVMulNoOverflow(cnt, _value))``, ``balances[sender] >= amount``;
* c4_wallet_*: solidity_examples/WalletLibrary.sol ``onlyowner`` lookups
  ``m_ownerIndex[uint(msg.sender)]`` (keccak mapping, line 391-397) with the
  transaction's sender among the LASER actors (transaction/symbolic.py:29-40,210-212);
* unsat_*: the reference tests' UNSAT shapes (tests/laser/keccak_tests.py:110-124,
  tests/laser/state/calldata_test.py:62-91).

Each file starts with ``; expect: sat|unsat``.  Run: python tests/make_solver_log_corpus.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mythril_amd.ir import Ctx  # noqa: E402
from mythril_amd.smt2 import to_smt2  # noqa: E402
from tests.mythril_shapes import KeccakManager, calldata_load, calldata_word  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "solver_log")
ACTORS = [0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE, 0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF,
          0xAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAA]


def tx_setup(c, tx="1"):
    s = c.var(f"sender_{tx}", 256)
    return s, [c.app("or", *[c.app("=", s, c.const(a, 256)) for a in ACTORS])]


def selector(c, tx, sel):
    return c.app("=", c.app("extract", calldata_word(c, tx, 0), params=(255, 224)), c.const(sel, 32))


def storage_at(c, km, key, slot, name="Storage[0x6f]"):
    h = km.create_keccak(c.app("concat", key, c.const(slot, 256)))
    return c.app("select", c.array(name, 256, 256), h)


def c2_token(underflow=True):
    c = Ctx()
    km = KeccakManager(c)
    sender, conj = tx_setup(c)
    value = calldata_word(c, "1", 36)
    bal = storage_at(c, km, sender, 0)
    conj += [selector(c, "1", 0xA9059CBB), c.app("bvule", c.const(68, 256), c.var("1_calldatasize", 256)),
             c.app("bvult", c.var("1_calldatasize", 256), c.const(1 << 12, 256))]
    # SWC-101: Not(BVSubNoUnderflow(bal, value)) == value >u bal
    conj.append(c.app("bvugt", value, bal) if underflow else c.app("bvule", value, bal))
    conj.append(km.create_conditions())
    return c, conj


def c3_bec():
    c = Ctx()
    km = KeccakManager(c)
    sender, conj = tx_setup(c)
    off = calldata_word(c, "1", 4)          # head of _receivers: offset of the array
    start = c.app("bvadd", c.const(4, 256), off)
    cnt = c.app("concat", *[calldata_load(c, "1", c.app("bvadd", start, c.const(i, 256))) for i in range(32)])
    value = calldata_word(c, "1", 36)
    amount = c.app("bvmul", cnt, value)
    bal = storage_at(c, km, sender, 3)
    conj += [selector(c, "1", 0x83F12FEC),
             c.app("bvugt", cnt, c.const(0, 256)), c.app("bvule", cnt, c.const(20, 256)),
             c.app("bvugt", value, c.const(0, 256)), c.app("bvuge", bal, amount),
             c.app("not", c.app("bvumul_noovfl", cnt, value)),
             c.app("bvult", c.var("1_calldatasize", 256), c.const(1 << 12, 256)),
             km.create_conditions()]
    return c, conj


def c4_wallet(owner=True):
    c = Ctx()
    km = KeccakManager(c)
    sender, conj = tx_setup(c)
    idx = storage_at(c, km, sender, 0x103, name="Storage[0x4c]")
    conj += [selector(c, "1", 0xCBF0B0C0), c.app("bvule", c.const(36, 256), c.var("1_calldatasize", 256))]
    conj.append(c.app("bvugt", idx, c.const(0, 256)) if owner else
                c.app("and", c.app("bvugt", idx, c.const(0, 256)), c.app("=", idx, c.const(0, 256))))
    conj.append(km.create_conditions())
    return c, conj


def unsat_keccak_number():
    c = Ctx()
    km = KeccakManager(c)
    o = km.create_keccak(c.var("a", 160))
    return c, [km.create_conditions(), c.app("=", c.const(10, 256), o)]


def unsat_calldata_bound():
    c = Ctx()
    v = calldata_load(c, "0", c.const(51, 256))
    return c, [c.app("=", v, c.const(1, 8)), c.app("=", c.var("0_calldatasize", 256), c.const(50, 256))]


CORPUS = {
    "c2_token_transfer_underflow": (lambda: c2_token(True), "sat"),
    "c2_token_transfer_ok": (lambda: c2_token(False), "sat"),
    "c3_bec_batchtransfer_overflow": (c3_bec, "sat"),
    "c4_wallet_onlyowner": (lambda: c4_wallet(True), "sat"),
    "c4_wallet_contradiction": (lambda: c4_wallet(False), "unsat"),
    "unsat_keccak_equals_10": (unsat_keccak_number, "unsat"),
    "unsat_calldata_out_of_bounds": (unsat_calldata_bound, "unsat"),
}


def main():
    os.makedirs(OUT, exist_ok=True)
    for name, (make, expect) in CORPUS.items():
        c, conj = make()
        with open(os.path.join(OUT, name + ".smt2"), "w") as f:
            f.write(f"; expect: {expect}\n; synthetic --solver-log dump (tests/make_solver_log_corpus.py)\n")
            f.write(to_smt2(conj))
        print(name, expect)


if __name__ == "__main__":
    main()
