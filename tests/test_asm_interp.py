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
    # every listed opcode has a handler label, and the introspection block
    # reports an offset for all 128 opcodes (handler or Lunsup)
    for o in isa.ASM_OPCODES:
        assert f"Lh_{o}_%=:" in txt, o
    # (twice: the wide and the narrow layout's interpreter)
    assert txt.count("- Lpc0_%=) >> 2)") == 2 * (128 + len(isa.ASM_FUSED))   # and every fused handler's
    for k in range(len(isa.ASM_FUSED)):
        assert f"Lf{k}_%=:" in txt
    assert "s_branch Lh_" not in txt          # one jump per dispatch: no table of branches


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
    bad = [f for f, p in progs if not isa.asm_eligible(p.code, p.leaves, p.consts)]
    assert not bad, bad
    assert len(progs) >= 170


def _predecode(code, consts):
    """mw_asm_predecode (mw_validate.cpp) through the library, on the CPU."""
    import ctypes

    import numpy as np

    from mythril_amd.runtime import LIB_PATH
    lib = ctypes.CDLL(LIB_PATH)
    f = lib.mw_asm_predecode
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                  ctypes.c_void_p, ctypes.c_void_p]
    code = np.ascontiguousarray(code, dtype=np.uint32)
    consts = np.ascontiguousarray(consts, dtype=np.uint32)
    out = np.zeros_like(code)
    nk = np.full(isa.ASM_NK, 0xDEAD, dtype=np.uint32)
    rc = f(code.ctypes.data, code.size, consts.ctypes.data, consts.size, HOFF.ctypes.data, out.ctypes.data,
           nk.ctypes.data)
    return (out.reshape(-1, 4), nk) if rc == 0 else (None, None)


# stand-in handler word offsets (the kernel reports the real ones at mg_init):
# the 128 opcodes', then the fused handlers'
HOFF = __import__("numpy").arange(1000, 1000 + (128 + len(isa.ASM_FUSED)) * 7, 7, dtype="uint32")


def test_predecode_operand_layout():
    """The asm engine's copy of the code: word 0 -> width | FLAG_CHAIN at bit 15
    | the opcode's handler word offset (one-jump dispatch), word 1 -> a [15:0]
    | dst [31:16] with dst the written register's index (N slot, W slot x 8),
    W register operands -> slot x 8, N register operands and W constants
    unchanged, N constants -> the index of their VGPR above the N file
    (176 + k, the value in table slot k), a W_CDINS index constant below
    0x4000 -> 0x4000 | index, and N_ADD's word 3 -> its width mask."""
    e = isa.encode
    consts = [0] * 17
    consts[0], consts[8], consts[16] = 0x24, 0x5000, 0x77   # two 256-bit constants, one narrow
    code = (e("N_ADD", 8, isa.encode_dst("N", 37), 3, isa.KBIT | 16)
            + e("W_ADD", 256, isa.encode_dst("W", 5), 2, isa.KBIT | 0)
            + e("N_ULT", 256, isa.encode_dst("N", 4), 6, 1)
            + e("W_ITE", 256, isa.encode_dst("W", 1), 3, 4, 9)
            + e("W_CDINS", 256, isa.encode_dst("W", 2), 2, 1, isa.KBIT | 0, imm=7 | (8 << 16))
            + e("W_CDINS", 256, isa.encode_dst("W", 2), 2, 1, isa.KBIT | 8, imm=7)
            + e("N_EQN", 8, isa.encode_dst("N", 5), isa.KBIT | 0, isa.KBIT | 16)
            + e("END", 0, isa.encode_dst(None)))
    o, nk = _predecode(code, consts)
    src = __import__("numpy").asarray(code, dtype="uint32").reshape(-1, 4)
    want0 = (src[:, 0] & 0xFFFF0000) | HOFF[src[:, 0] & 0x7F] | (((src[:, 0] >> 8) & isa.FLAG_CHAIN) << 15)
    assert (o[:, 0] == want0).all()
    assert o[0, 3] == 0xFF and (o[1:, 3] == src[1:, 3]).all()       # N_ADD: the 8-bit mask
    assert o[0, 1] == 3 | (37 << 16) and o[0, 2] == 176 + 0          # narrow constant 0x77 -> NK slot 0
    assert list(nk[:2]) == [0x77, 0x24] and not nk[2:].any()
    assert o[6, 1] == (176 + 1) | (5 << 16) and o[6, 2] == 176 + 0  # 0x24 (narrow use) -> slot 1, 0x77 reused
    assert o[1, 1] == 16 | (40 << 16) and o[1, 2] == isa.KBIT | 0
    assert o[2, 1] == 48 | (4 << 16) and o[2, 2] == 8
    assert o[3, 1] == 24 | (8 << 16) and o[3, 2] == 32 | (9 << 16)   # c is the N condition
    assert o[4, 2] == 8 | ((0x4000 | 0x24) << 16)
    assert o[5, 2] == 8 | ((isa.KBIT | 8) << 16)                          # 0x5000: stays a constant


def test_predecode_narrow_constant_bound():
    """More distinct narrow constants than the asm interpreter's VGPRs hold:
    predecode refuses (the program runs on the compiled interpreter) and the
    host mirror agrees."""
    e = isa.encode
    n = isa.ASM_NK + 1
    consts = list(range(100, 100 + n))
    code = []
    for k in range(n):
        code += e("N_ADD", 16, isa.encode_dst("N", k % 30), k % 30, isa.KBIT | k)
    code += e("END", 0, isa.encode_dst(None))
    o, _ = _predecode(code, consts)
    assert o is None
    leaves = []
    assert not isa.asm_eligible(code, leaves, consts)
    assert isa.asm_eligible(code[:-8 * 4] + e("END", 0, isa.encode_dst(None)), leaves, consts)
    assert len(isa.asm_narrow_constants(code, consts)) == n


def test_predecode_fused_sequences():
    """The first instruction of every fused-sequence match (left to right,
    longest first) jumps to that sequence's handler (offset entry 128 + k);
    the rest of the match keeps its own words, and the match agrees with
    isa.asm_fused_dispatch."""
    import numpy as np
    e = isa.encode
    N = lambda k: isa.encode_dst("N", k)   # noqa: E731
    code = (e("N_SLT", 1, N(1), 2, 3) + e("LEAF_N", 8, N(4), imm=0) + e("N_ITE", 8, N(5), 4, 6, 1)
            + e("N_SHLI", 32, N(6), 5, imm=8)                                  # the 4-op calldata byte
            + e("N_SLT", 1, N(1), 2, 3) + e("LEAF_N", 8, N(4), imm=1) + e("N_ITE", 8, N(5), 4, 6, 1)
            + e("N_ADD", 8, N(7), 1, 2)                                        # 3-op prefix, then none
            + e("N_XOR", 1, N(8), 1, 2) + e("CHECK", 0, isa.encode_dst(None), 8)
            + e("END", 0, isa.encode_dst(None)))
    o, _ = _predecode(code, [0])
    src = np.asarray(code, dtype="uint32").reshape(-1, 4)
    plain = (src[:, 0] & 0xFFFF0000) | HOFF[src[:, 0] & 0x7F]
    fused = {i: k for i, k in isa.asm_fused_dispatch(code) if k is not None}
    seq = lambda *t: isa.ASM_FUSED.index(tuple(t))   # noqa: E731
    assert fused == {0: seq("N_SLT", "LEAF_N", "N_ITE", "N_SHLI"), 4: seq("N_SLT", "LEAF_N", "N_ITE"),
                     8: seq("N_XOR", "CHECK")}
    for i in range(len(src)):
        want = (plain[i] & 0xFFFF8000) | HOFF[128 + fused[i]] if i in fused else plain[i]
        assert o[i, 0] == want, i


def _predecode_layout(code, consts, nk_index, nk_max, nfile):
    import ctypes

    import numpy as np

    from mythril_amd.runtime import LIB_PATH
    f = ctypes.CDLL(LIB_PATH).mw_asm_predecode_layout
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
    code = np.ascontiguousarray(code, dtype=np.uint32)
    consts = np.ascontiguousarray(consts, dtype=np.uint32)
    out = np.zeros_like(code)
    nk = np.full(isa.ASM_NK, 0xDEAD, dtype=np.uint32)
    rc = f(code.ctypes.data, code.size, consts.ctypes.data, consts.size, HOFF.ctypes.data, out.ctypes.data,
           nk.ctypes.data, nk_index, nk_max, nfile)
    return rc, out.reshape(-1, 4), nk


def test_narrow_layout_predecode():
    """Round 5: the asm interpreter's second kernel holds a 24-slot N file and
    14 narrow constants at v64 + 88 (asmgen.variant("narrow")).  A program is
    predecoded for it only when every N register lies below 24 (else -2: the
    wide kernel runs it); its narrow constants then name VGPR 88 + k, and the
    rest of the copy is the wide predecode's."""
    from mythril_amd import asmgen
    nv = asmgen.variant("narrow")
    assert (nv.NFILE, nv.NK_INDEX, nv.NKN, nv.NVGPR) == (24, 88, 14, 166)
    assert nv.XA == 96 and nv.T + 8 == nv.NK0 and asmgen.XA == 136
    e = isa.encode
    consts = [0] * 9
    consts[8] = 0x77
    code = (e("N_ADD", 8, isa.encode_dst("N", 7), 3, isa.KBIT | 8) + e("N_ULT", 8, isa.encode_dst("N", 23), 7, 3)
            + e("END", 0, isa.encode_dst(None)))
    rc, o, nk = _predecode_layout(code, consts, 88, 14, 24)
    assert rc == 0 and o[0, 2] == 88 and nk[0] == 0x77
    wide, _ = _predecode(code, consts)
    assert (o[:, 0] == wide[:, 0]).all() and (o[1:, 1:] == wide[1:, 1:]).all()
    high = code[:-4] + e("N_NOT", 8, isa.encode_dst("N", 24), 23) + e("END", 0, isa.encode_dst(None))
    assert _predecode_layout(high, consts, 88, 14, 24)[0] == -2
    assert _predecode_layout(high, consts, 176, 16, 0)[0] == 0      # no file bound: the wide layout
    many = [0] * 15 + list(range(100, 115))
    wide_k = sum((e("N_ADD", 8, isa.encode_dst("N", 1), 0, isa.KBIT | (15 + i)) for i in range(15)), [])
    assert _predecode_layout(wide_k + e("END", 0, isa.encode_dst(None)), many, 88, 14, 24)[0] == -1


def test_corpus_mostly_fits_the_narrow_layout():
    """The LASER corpus: most programs keep their N registers below 24 slots."""
    progs = [p for f, p in _corpus_programs() if ".gz" in f]
    fit = sum(_predecode_layout(p.code, p.consts, 88, 14, 24)[0] == 0 for p in progs)
    assert fit >= 0.9 * len(progs), (fit, len(progs))
