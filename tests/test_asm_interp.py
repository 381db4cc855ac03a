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
    # every fused handler's too, per bank, in each of the three layouts'
    # interpreters (wide, narrow, quarter)
    assert txt.count("- Lpc0_%=) >> 2)") == 3 * 2 * (128 + len(isa.ASM_FUSED))
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


# a stand-in introspection table (the kernel reports the real one at mg_init):
# bank A's handler word offsets (the 128 opcodes', then the fused handlers'),
# bank B's, then the interpreter's base address (low, high word)
NH = 128 + len(isa.ASM_FUSED)
LPC0 = 0x7F001000
HOFF = __import__("numpy").concatenate([__import__("numpy").arange(1000, 1000 + NH * 7, 7),
                                        __import__("numpy").arange(9000, 9000 + NH * 5, 5),
                                        [LPC0, 0x7FFF]]).astype("uint32")


def _target(i, h):
    """word 0 of instruction i dispatching to handler entry h: the handler's
    absolute address (low word) in bank i & 1"""
    return LPC0 + 4 * int(HOFF[(i & 1) * NH + h])


def test_predecode_operand_layout():
    """The asm engine's copy of the code: word 0 -> the low word of the
    opcode's handler address in the instruction's bank (i & 1: a move and a
    jump dispatch it), word 1 -> a [15:0] | dst [23:16] | width - 1 [31:24]
    with dst the written register's index (N slot, W slot x 8),
    W register operands -> slot x 8, N register operands and W constants
    unchanged, N constants -> the index of their VGPR above the N file
    (176 + k, the value in table slot k), a W_CDINS index constant below
    0x4000 -> 0x4000 | index, a chained W_CDINS's FLAG_CHAIN -> bit 31 of its
    immediate, and N_ADD's word 3 -> its width mask."""
    e = isa.encode
    consts = [0] * 17
    consts[0], consts[8], consts[16] = 0x24, 0x5000, 0x77   # two 256-bit constants, one narrow
    code = (e("N_ADD", 8, isa.encode_dst("N", 37), 3, isa.KBIT | 16)
            + e("W_ADD", 256, isa.encode_dst("W", 5), 2, isa.KBIT | 0)
            + e("N_ULT", 256, isa.encode_dst("N", 4), 6, 1)
            + e("W_ITE", 256, isa.encode_dst("W", 1), 3, 4, 9)
            + e("W_CDINS", 256, isa.encode_dst("W", 2), 2, 1, isa.KBIT | 0, imm=7 | (8 << 16), flags=isa.FLAG_CHAIN)
            + e("W_CDINS", 256, isa.encode_dst("W", 2), 2, 1, isa.KBIT | 8, imm=7)
            + e("N_EQN", 8, isa.encode_dst("N", 5), isa.KBIT | 0, isa.KBIT | 16)
            + e("END", 0, isa.encode_dst(None)))
    o, nk = _predecode(code, consts)
    src = __import__("numpy").asarray(code, dtype="uint32").reshape(-1, 4)
    assert [int(x) for x in o[:, 0]] == [_target(i, int(op) & 0x7F) for i, op in enumerate(src[:, 0])]
    assert o[0, 3] == 0xFF and (o[[1, 2, 5, 6, 7], 3] == src[[1, 2, 5, 6, 7], 3]).all()   # N_ADD: the mask
    assert o[3, 3] == 9                                              # W_ITE: c (no immediate) in word 3 too
    assert o[4, 3] == src[4, 3] | 0x80000000                         # the chain flag
    w1 = lambda lo, d, w: lo | (d << 16) | ((w - 1) << 24)           # noqa: E731
    assert o[0, 1] == w1(3, 37, 8) and o[0, 2] == 176 + 0            # narrow constant 0x77 -> NK slot 0
    assert list(nk[:2]) == [0x77, 0x24] and not nk[2:].any()
    assert o[6, 1] == w1(176 + 1, 5, 8) and o[6, 2] == 176 + 0       # 0x24 (narrow use) -> slot 1, 0x77 reused
    assert o[1, 1] == w1(16, 40, 256) and o[1, 2] == isa.KBIT | 0
    assert o[2, 1] == w1(48, 4, 256) and o[2, 2] == 8
    assert o[3, 1] == w1(24, 8, 256) and o[3, 2] == 32 | (9 << 16)   # c is the N condition
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
    longest first) jumps to that sequence's handler (entry 128 + k of its bank);
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
    plain = [_target(i, int(op) & 0x7F) for i, op in enumerate(src[:, 0])]
    fused = {i: k for i, k in isa.asm_fused_dispatch(code) if k is not None}
    seq = lambda *t: isa.ASM_FUSED.index(tuple(t))   # noqa: E731
    assert fused == {0: seq("N_SLT", "LEAF_N", "N_ITE", "N_SHLI"), 4: seq("N_SLT", "LEAF_N", "N_ITE"),
                     8: seq("N_XOR", "CHECK")}
    for i in range(len(src)):
        want = _target(i, 128 + fused[i]) if i in fused else plain[i]
        assert o[i, 0] == want, i


def test_predecode_refuses_a_carry_into_the_high_word():
    """The kernel keeps one high word for every handler address (s93): code
    whose handlers straddle a 4 GiB boundary is not predecoded (-3; the
    compiled interpreter runs it)."""
    import numpy as np
    global HOFF
    code = isa.encode("N_ADD", 8, isa.encode_dst("N", 1), 2, 3) + isa.encode("END", 0, isa.encode_dst(None))
    saved = HOFF
    try:
        HOFF = saved.copy()
        HOFF[2 * NH] = np.uint32(0xFFFFFFFF - 4 * 1000)
        rc, _, _ = _predecode_layout(code, [0], 176, 16, 0)
        assert rc == -3
    finally:
        HOFF = saved
    assert _predecode_layout(code, [0], 176, 16, 0)[0] == 0


def _predecode_layout(code, consts, nk_index, nk_max, nfile, wfile=0):
    import ctypes

    import numpy as np

    from mythril_amd.runtime import LIB_PATH
    f = ctypes.CDLL(LIB_PATH).mw_asm_predecode_layout
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                  ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                  ctypes.c_uint32]
    code = np.ascontiguousarray(code, dtype=np.uint32)
    consts = np.ascontiguousarray(consts, dtype=np.uint32)
    out = np.zeros_like(code)
    nk = np.full(isa.ASM_NK, 0xDEAD, dtype=np.uint32)
    rc = f(code.ctypes.data, code.size, consts.ctypes.data, consts.size, HOFF.ctypes.data, out.ctypes.data,
           nk.ctypes.data, nk_index, nk_max, nfile, wfile)
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


def test_quarter_layout_predecode():
    """Round 5: the third asm kernel (asmgen.variant("quarter")) holds 5 W
    slots, 16 N slots and 4 narrow constants in 124 VGPRs (four waves per
    SIMD).  A program is predecoded for it only when every W register
    (operand or result) lies below 5 and every N register below 16 (else -2)."""
    from mythril_amd import asmgen
    qv = asmgen.variant("quarter")
    assert (qv.WFILE, qv.NFILE, qv.N0, qv.NK_INDEX, qv.NKN, qv.NVGPR) == (5, 16, 40, 80, 4, 124)
    e = isa.encode
    consts = [0] * 9
    consts[8] = 0x77
    ok = (e("LEAF_W", 256, isa.encode_dst("W", 3), imm=0) + e("W_ADD", 256, isa.encode_dst("W", 1), 3, 3)
          + e("N_EQ", 256, isa.encode_dst("N", 15), 1, isa.KBIT | 0) + e("END", 0, isa.encode_dst(None)))
    rc, o, _ = _predecode_layout(ok, consts, 80, 4, 16, 5)
    assert rc == 0 and o[1, 1] & 0xFF == 24 and (o[1, 1] >> 16) & 0xFF == 8      # a = W3 x 8, dst = W1 x 8
    wdst = ok[:-4] + e("MOV_W", 256, isa.encode_dst("W", 5), 1) + e("END", 0, isa.encode_dst(None))
    wsrc = ok[:-4] + e("W_NOT", 256, isa.encode_dst("W", 0), 6) + e("END", 0, isa.encode_dst(None))
    nsrc = ok[:-4] + e("N_NOT", 8, isa.encode_dst("N", 2), 16) + e("END", 0, isa.encode_dst(None))
    for bad in (wdst, wsrc, nsrc):
        assert _predecode_layout(bad, consts, 80, 4, 16, 5)[0] == -2
        assert _predecode_layout(bad, consts, 88, 14, 24, 0)[0] == 0      # the narrow layout holds them


def test_corpus_fits_the_quarter_layout_in_part():
    """About half of the LASER corpus (as compiled) keeps its registers in the
    quarter layout's files."""
    progs = [p for f, p in _corpus_programs() if ".gz" in f]
    fit = sum(_predecode_layout(p.code, p.consts, 80, 4, 16, 5)[0] == 0 for p in progs)
    assert fit >= 0.35 * len(progs), (fit, len(progs))


def test_predecode_chains_check_impeq_runs():
    """Round 5: a CHECK_IMPEQ followed by another gets bit 31 of word 3 (its c
    field in the low bits): the handler takes the next one itself."""
    e = isa.encode
    N = lambda k: isa.encode_dst("N", k)   # noqa: E731
    none = isa.encode_dst(None)
    code = (e("N_EQN", 8, N(1), 2, 3) + e("CHECK_IMPEQ", 0, none, 1, 4, 5) + e("CHECK_IMPEQ", 0, none, 1, 6, 7)
            + e("CHECK_IMPEQ", 0, none, 1, 8, 9) + e("CHECK", 0, none, 1) + e("CHECK_IMPEQ", 0, none, 1, 2, 3)
            + e("END", 0, none))
    o, _ = _predecode(code, [0])
    assert [int(x) >> 31 for x in o[:, 3]] == [0, 1, 1, 0, 0, 0, 0]
    assert [int(x) & 0xFFFF for x in o[1:4, 3]] == [5, 7, 9]      # c in the low bits, as before


def test_predecode_chains_keyed_checks():
    """CHECK_IMPEQK keeps its premise constant whole in word 3: a keyed check
    followed by another gets bit 31 of word 1 instead (above the width, which
    its handler does not read), and a following unkeyed check ends the chain."""
    e = isa.encode
    none = isa.encode_dst(None)
    K = 0x7FFFFFFF
    code = (e("CHECK_IMPEQK", 8, none, 1, 4, 5, imm=0x10020) + e("CHECK_IMPEQK", 255, none, 1, 6, 7, imm=K)
            + e("CHECK_IMPEQK", 200, none, 1, 8, 9, imm=3) + e("CHECK_IMPEQ", 0, none, 1, 2, 3)
            + e("CHECK_IMPEQK", 8, none, 1, 2, 3, imm=4) + e("END", 0, none))
    o, _ = _predecode(code, [0])
    assert [int(o[i, 1]) >> 31 for i in (0, 1, 2, 4)] == [1, 1, 0, 0]   # (the other rows' width bits)
    assert [int(x) for x in o[:3, 3]] == [0x10020, K, 3]         # the premise constants, whole
    assert [int(x) & 0xFF for x in o[:3, 1]] == [1, 1, 1]           # the key's register
    assert [int(x) for x in o[:3, 2]] == [4 | 5 << 16, 6 | 7 << 16, 8 | 9 << 16]
