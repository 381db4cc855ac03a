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
                                   "underflow_t3_send_send_balance_q37_sat.smt2.gz"])
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
