"""CPU checks of the threaded-dispatch asm interpreter:
the committed mw_asm_interp.inc is what tools/gen_asm_interp.py generates, the
host and device opcode lists agree, and the Mythril-shaped corpora (solver-log
C2-C4 queries and the LASER corpus) are eligible for it.  tests/test_gpu_asm.py
checks its results on the device."""
import os
import re
import subprocess
import sys

from mythril_amd import isa

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "mythril_amd", "csrc", "mw_asm_interp.inc")


def test_generated_asm_is_current():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_asm_interp.py"), "--check"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def test_opcode_lists_agree():
    txt = open(INC).read()
    ops = re.search(r"#define MW_ASM_OPCODES (.*)", txt).group(1).split(", ")
    assert [o[3:] for o in ops] == isa.ASM_OPCODES
    kinds = [int(k) for k in re.search(r"#define MW_ASM_LEAF_KINDS (.*)", txt).group(1).split(", ")]
    assert kinds == isa.ASM_LEAF_KINDS
    # every listed opcode has a handler label, and the dispatch table has 128 entries
    for o in isa.ASM_OPCODES:
        assert f"Lh_{o}_%=:" in txt, o
    assert txt.count("s_branch Lh_") + txt.count("s_branch Lunsup_%=") >= 128


def _corpus_programs():
    from mythril_amd.engine import prepare
    from mythril_amd.smt2 import parse_file
    out = []
    for d in ("solver_log", "laser"):
        base = os.path.join(ROOT, "tests", "golden", d)
        for f in sorted(os.listdir(base)):
            if f.endswith(".smt2") or f.endswith(".smt2.gz"):
                s = parse_file(os.path.join(base, f))
                out.append((f, prepare(s.asserts, s.ctx).program))
    return out


def test_mythril_corpora_are_asm_eligible():
    progs = _corpus_programs()
    bad = [f for f, p in progs if not isa.asm_eligible(p.code, p.leaves)]
    assert not bad, bad
    assert len(progs) >= 170
