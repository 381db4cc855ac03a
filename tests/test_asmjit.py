"""CPU checks of the assembled kernels (mythril_amd/asmjit.py): the template
exists and carries its marker, and every corpus program assembles (llvm-mc +
ld.lld, here on the CPU) into a code object exporting the kernel and its
signature word.  tests/test_gpu_asmjit.py runs them on the device."""
import os
import subprocess

import pytest

from mythril_amd import asmgen, asmjit
from mythril_amd.jit import signature

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_template_is_built_and_marked():
    assert asmjit.available(), "run python -m mythril_amd.build"
    text = asmjit.TEMPLATE.read_text()
    assert text.count(asmgen.MARKER) == 1
    assert asmjit.TEMPLATE_NAME in text


@pytest.mark.parametrize("which", ["c2_token_transfer_underflow.smt2", "c4_wallet_onlyowner.smt2",
                                   "underflow_t3_send_send_balance_q41_sat.smt2.gz",
                                   "flag_array_t2_extract_money_q15_sat.smt2.gz"])   # W_UDIV: the loop
def test_corpus_programs_assemble(which, tmp_path):
    from mythril_amd.engine import prepare
    from mythril_amd.smt2 import parse_file
    d = "laser" if which.endswith(".gz") else "solver_log"
    s = parse_file(os.path.join(ROOT, "tests", "golden", d, which))
    p = prepare(s.asserts, s.ctx).program
    image, name, _ = asmjit.assemble(p, cache=False)
    assert name == f"mwa_{signature(p):016x}"
    co = tmp_path / "k.hsaco"
    co.write_bytes(image)
    syms = subprocess.run([str(asmjit.LLVM_BIN / "llvm-readelf"), "-s", str(co)], capture_output=True,
                          text=True).stdout
    assert f" {name}\n" in syms and f" {name}_sig\n" in syms and f" {name}.kd\n" in syms


def test_static_body_has_no_dispatch_or_indexing():
    """Straight-line: no instruction fetch and no table jump; operands are
    literal registers and constants (a few handlers still index a limb by a
    width-derived amount)."""
    from mythril_amd.engine import prepare
    from mythril_amd.smt2 import parse_file
    s = parse_file(os.path.join(ROOT, "tests", "golden", "solver_log", "c2_token_transfer_underflow.smt2"))
    p = prepare(s.asserts, s.ctx).program
    body = "\n".join(asmgen.static_body(p.code, p.consts, p.leaves))
    for bad in ("s_load_dwordx4", "Ltab", "s_setpc_b64 s[92:93]"):
        assert bad not in body, bad
    assert body.count("s_set_gpr_idx_on") < 10


def test_random_programs_assemble():
    """Every handled opcode through the static handlers, constant folding and
    dead-code passes, with and without pools: llvm-mc accepts the result
    (operand encodings, the constant bus).  Verdicts are checked on the GPU
    (tests/test_gpu_asmjit.py)."""
    if not asmjit.available():
        pytest.skip("no assembled-kernel template (python -m mythril_amd.build)")
    from mythril_amd import isa
    from mythril_amd.engine import prepare
    from tests.test_gpu_asm import _random_supported_dag
    n = 0
    for seed in range(9000, 9016):
        c, conj = _random_supported_dag(seed)
        for pools in (False, True):
            p = prepare(conj, c, use_pools=pools).program
            if not isa.asm_eligible(p.code, p.leaves, p.consts):
                continue
            image, name, _ = asmjit.assemble(p, cache=False)
            assert image[:4] == b"\x7fELF" and name == asmjit.kernel_name(p)
            n += 1
    assert n >= 16


def test_const_fold_rules():
    """The constant-operand peephole keeps each encoding legal: a literal only
    in a VOP2 / VOPC src0 and never beside a carry-in, src1 stays a VGPR."""
    body = ["v_mov_b32_e32 v152, 0xaffeaffe", "v_mov_b32_e32 v153, 0", "v_mov_b32_e32 v154, 0x80000000",
            "v_xor_b32_e32 v184, v176, v152", "v_xor_b32_e32 v185, v177, v153",
            "v_sub_co_u32_e32 v186, vcc, v176, v152", "v_subb_co_u32_e32 v187, vcc, v154, v177, vcc",
            "v_subb_co_u32_e32 v188, vcc, v153, v177, vcc", "v_cmp_lt_u32_e32 vcc, v176, v152",
            "v_xor_b32_e32 v189, s74, v152"]
    out = asmgen.const_fold(body)
    assert out[3] == "v_xor_b32_e32 v184, 0xaffeaffe, v176"
    assert out[4] == "v_mov_b32_e32 v185, v177"
    assert out[5] == "v_subrev_co_u32_e32 v186, vcc, 0xaffeaffe, v176"
    assert out[6] == "v_subb_co_u32_e32 v187, vcc, v154, v177, vcc"      # literal + vcc: unchanged
    assert out[7] == "v_subb_co_u32_e32 v188, vcc, 0, v177, vcc"         # inline constant: allowed
    assert out[8] == "v_cmp_gt_u32_e32 vcc, 0xaffeaffe, v176"
    assert out[9] == "v_xor_b32_e32 v189, s74, v152"                     # src0 an SGPR: no swap


def test_dead_code_liveness():
    """Backward liveness of asmgen.dead_code: a copy nobody reads goes, a copy
    read after a forward skip's label stays, file registers are dead at the
    exit while the template's (v160..v167) are live, a call keeps v128 and up
    live, an s_set_gpr_idx region reads everything, and registers read before
    any write come back as live-in."""
    XA, T = asmgen.XA, asmgen.T
    body = [
        f"v_mov_b32_e32 v{XA}, v3",                 # dead: overwritten below before any read
        f"v_mov_b32_e32 v{XA}, v4",
        f"v_mov_b32_e32 v{T}, v{XA}",               # read after the label: stays
        "s_cbranch_vccz LSx1_%=",
        "v_mov_b32_e32 v5, 0",                      # dead at the exit (file register)
        "LSx1_%=:",
        f"v_add_u32_e32 v162, v{T}, v162",          # ALIVE: live at exit
        "v_mov_b32_e32 v6, v7",                     # dead
        "s_setpc_b64 s[40:41]",
    ]
    out, live_in = asmgen.dead_code(body)
    assert f"v_mov_b32_e32 v{XA}, v3" not in out
    assert f"v_mov_b32_e32 v{T}, v{XA}" in out and f"v_mov_b32_e32 v{XA}, v4" in out
    assert "v_mov_b32_e32 v5, 0" not in out and "v_mov_b32_e32 v6, v7" not in out
    assert 4 in live_in and 3 not in live_in and 7 not in live_in
    # an unknown call: every register from v128 up is live across it
    out, _ = asmgen.dead_code([f"v_mov_b32_e32 v{T + 1}, 5", "s_swappc_b64 s[68:69], s[44:45]",
                               "s_setpc_b64 s[40:41]"])
    assert f"v_mov_b32_e32 v{T + 1}, 5" in out
    # the Philox subroutine writes T..T+7 and reads only the candidate index
    out, _ = asmgen.dead_code([f"v_mov_b32_e32 v{T + 1}, 5", f"v_mov_b32_e32 v{XA}, 5",
                               "s_swappc_b64 s[70:71], s[48:49]", f"v_mov_b32_e32 v{T + 2}, v{XA}",
                               f"v_add_u32_e32 v162, v{T + 2}, v162", "s_setpc_b64 s[40:41]"])
    assert f"v_mov_b32_e32 v{T + 1}, 5" not in out      # overwritten by the subroutine
    assert f"v_mov_b32_e32 v{XA}, 5" in out             # read after the call
    # an indexed region reads everything
    out, live_in = asmgen.dead_code(["v_mov_b32_e32 v9, 1", "s_set_gpr_idx_on s19, gpr_idx(SRC0)",
                                     "v_mov_b32_e32 v136, v0", "s_set_gpr_idx_off", "s_setpc_b64 s[40:41]"])
    assert "v_mov_b32_e32 v9, 1" in out and 0 in live_in


def test_one_entry_pool_leaves_fold():
    """C4's calldata bytes have one-entry pools: with the pool words in hand
    the static body reads no pool entry for them and loads the constant."""
    from mythril_amd.engine import prepare
    from mythril_amd.smt2 import parse_file
    s = parse_file(os.path.join(ROOT, "tests", "golden", "solver_log", "c4_wallet_onlyowner.smt2"))
    p = prepare(s.asserts, s.ctx).program
    nl = asmgen.lds_spill_words(p.n_spill, len(p.pool))
    without = asmgen.static_body(p.code, p.consts, p.leaves, nlds=nl)
    folded = asmgen.static_body(p.code, p.consts, p.leaves, nlds=nl, pool=p.pool)
    reads = lambda body: sum(1 for ln in body if ln.startswith("ds_read"))   # noqa: E731
    assert reads(folded) < reads(without)
    assert sum(1 for ln in folded if ln.startswith("v_")) < sum(1 for ln in without if ln.startswith("v_"))


def test_traced_programs_stay_on_the_interpreter():
    """STORE_W / STORE_N are asm-interpreter handlers only (trace rows of
    mg_eval_generated): a traced program is asm-eligible but never assembled."""
    from mythril_amd import isa
    from mythril_amd.compiler import compile_program
    from mythril_amd.ir import Ctx
    c = Ctx()
    x = c.var("x", 64)
    conj = [c.app("bvult", x, c.const(1000, 64))]
    traced = compile_program(conj, trace=[x])
    plain = compile_program(conj)
    assert isa.asm_eligible(traced.code, traced.leaves, traced.consts)
    assert not asmjit.eligible(traced)
    assert asmjit.eligible(plain)
    # and the generated interpreter has both handlers
    assert "Lh_STORE_W_" in "\n".join(asmgen.gen()) and "Lh_STORE_N_" in "\n".join(asmgen.gen())
