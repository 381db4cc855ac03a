"""The specialised kernels' column multiply (mw_jit.h mul8_cols).

CPU side: the asm in the header is what tools/gen_mul_cols.py generates, every
carry read sits two VALU instructions (or an s_nop's wait states) after its
write, and the emitter picks mul8_cols only for two register operands.  The
device check is tests/test_gpu_jit.py::test_mul_cols_against_oracle.
"""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def _header_columns() -> str:
    src = open(os.path.join(ROOT, "mythril_amd", "csrc", "mw_jit.h")).read()
    start = src.index("  // column 1\n")
    end = src.index("  r[6] = (u32)p;")
    return src[start:end].rstrip("\n")


def test_header_is_generated():
    import gen_mul_cols
    assert _header_columns() == gen_mul_cols.statements()


def test_carry_reads_respect_the_wait_states():
    import gen_mul_cols
    for k in range(1, 7):
        lines = gen_mul_cols.column(k, k <= 5)
        last_write = {}
        waits = 0          # wait states since the start (VALU = 1, s_nop n = n + 1)
        for ln in lines:
            m = re.match(r"s_nop (\d)", ln)
            if m:
                waits += int(m.group(1)) + 1
                continue
            if ln.startswith("v_addc_co_u32_e64"):
                s = re.findall(r"%\[(s\d)\]", ln)[-1]       # the carry-in
                assert waits - last_write[s] - 1 >= 2, (k, ln)
            dst = re.findall(r"%\[(s\d)\]", ln)[0]          # the carry-out written
            waits += 1
            last_write[dst] = waits - 1


def test_products_per_column():
    import gen_mul_cols
    for k in range(1, 7):
        lines = gen_mul_cols.column(k, k <= 5)
        mads = [ln for ln in lines if ln.startswith("v_mad_u64_u32")]
        assert len(mads) == k + 1
        pairs = {tuple(map(int, re.findall(r"%\[[ab](\d)\]", ln))) for ln in mads}
        assert pairs == {(i, k - i) for i in range(k + 1)}
        addcs = [ln for ln in lines if ln.startswith("v_addc")]
        assert len(addcs) == (0 if k == 6 else (1 if k == 1 else k + 1))


def test_emitter_uses_columns_for_register_operands(monkeypatch):
    from mythril_amd import jit
    from mythril_amd.compiler import compile_program
    from mythril_amd.ir import Ctx
    c = Ctx()
    x, y = c.var("x", 256), c.var("y", 256)
    conj = [c.app("=", c.app("bvmul", x, y), c.const(12, 256)),
            c.app("bvugt", c.app("bvmul", x, c.const(3, 256)), c.const(5, 256))]
    p = compile_program(conj)
    monkeypatch.setattr(jit, "MUL_COLS", True)
    src = jit.generate([p], ["t"])
    assert src.count("jit::w_mulv(") == 1 and src.count("jit::w_mul(") == 1
    monkeypatch.setattr(jit, "MUL_COLS", False)
    src = jit.generate([p], ["t"])
    assert "jit::w_mulv(" not in src and src.count("jit::w_mul(") == 2
