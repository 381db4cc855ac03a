"""Instruction-priced executed work (isa.executed_ops_per_eval, VERDICT r5
item 2): every opcode is priced, a congruence grid row costs one lookup, and
C3 - whose 68 grid rows stand for 2 176 pair checks - executes far less than
its DAG-priced ops_per_eval, so no engine's frac_peak exceeds 1 once the
smaller count is used (tools/config_bench.py)."""
import os

from mythril_amd import isa
from mythril_amd.engine import prepare
from mythril_amd.smt2 import parse_file

LOG = os.path.join(os.path.dirname(__file__), "golden", "solver_log")


def test_every_opcode_is_priced():
    for op in isa.OPCODES:
        for w in (1, 8, 32, 160, 256):
            assert isa.insn_ops(op, w) >= 0
    assert isa.insn_ops("CHECK_GRID", 8) < 32 * isa.insn_ops("CHECK_IMPEQK", 8)
    assert isa.insn_ops("W_MUL", 256) == 2 * 8 * 9
    assert isa.insn_ops("SPILL_N", 0) == isa.insn_ops("LEAF_W", 256) == 0


def test_c3_grid_rows_priced_as_executed():
    s = parse_file(os.path.join(LOG, "c3_bec_batchtransfer_overflow.smt2"))
    q = prepare(s.asserts, s.ctx)
    for p in (q.program, q.long_program):
        ex = isa.executed_ops_per_eval(p.code)
        rows = sum(1 for w in p.code[0::4] if int(w) & 0xFF == isa.OPCODES["CHECK_GRID"])
        assert rows >= 60
        assert ex < 0.3 * p.ops_per_eval, (ex, p.ops_per_eval)


def test_programs_without_grids_stay_near_the_dag_count():
    for f in ("c2_token_transfer_ok.smt2", "c4_wallet_onlyowner.smt2"):
        s = parse_file(os.path.join(LOG, f))
        p = prepare(s.asserts, s.ctx).program
        ex = isa.executed_ops_per_eval(p.code)
        assert 0.8 * p.ops_per_eval <= ex <= 1.3 * p.ops_per_eval, (f, ex, p.ops_per_eval)
