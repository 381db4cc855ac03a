"""Python mirror of ``csrc/mw_isa.h`` (kept in sync by tests/test_isa_sync.py)."""
from __future__ import annotations

NW = 8           # W file slots (8 x u32 limbs each)
NN = 64          # N file slots (1 x u32 each)
W_RESERVED = NW - 1   # interpreter write-back scratch slots, never allocated (mw_isa.h)
N_RESERVED = 31       # N slots 31 and 63
KBIT = 0x8000
LEAF_WORDS = 8
POOL_ENTRY_WORDS = 9       # wide leaves (width >= 32): flags + 8 limbs
POOL_NARROW_RANDOM = 0x80000000   # narrow leaves (width < 32): one word per entry


def pool_entry_words(width: int) -> int:
    """words per pool entry of a width-bit leaf (mw_isa.h MW_POOL_ENTRY_WORDS_OF)"""
    return 1 if width < 32 else POOL_ENTRY_WORDS
MAX_WIDTH = 256
NARROW_MAX = 32

LEAF_WIDTH, LEAF_KIND, LEAF_ID, LEAF_SHIFT, LEAF_BITS, LEAF_POOL, LEAF_INROW = range(7)

OPCODES = {
    "END": 0, "CHECK": 1, "LEAF_W": 2, "LEAF_N": 3, "STORE_W": 4, "STORE_N": 5,
    "SPILL_W": 6, "FILL_W": 7, "MOV_W": 8, "MOV_N": 9, "SPILL_N": 10, "FILL_N": 11, "CHECK_IMP": 12,
    "CHECK_IMPEQ": 13, "CHECK_IMPEQW": 14, "CHECK_IMPEQK": 15,
    "W_ADD": 16, "W_SUB": 17, "W_MUL": 18, "W_AND": 19, "W_OR": 20, "W_XOR": 21, "W_NOT": 22,
    "W_SHL": 23, "W_LSHR": 24, "W_ASHR": 25,
    "W_UDIV": 26, "W_UREM": 27, "W_SDIV": 28, "W_SREM": 29, "W_SMOD": 30,
    "W_ITE": 31, "W_SHLI": 32, "W_LSHRI": 33, "W_ZEXTN": 34, "W_SEXT": 35, "W_SEXTN": 36,
    "W_INSN": 37, "W_CDINS": 38, "CHECK_GRID": 39,
    "N_EXTRACTW": 48, "N_ULT": 49, "N_ULE": 50, "N_SLT": 51, "N_SLE": 52, "N_EQ": 53,
    "N_UMULNO": 54, "N_ADDC": 55,
    "N_ADD": 64, "N_SUB": 65, "N_MUL": 66, "N_AND": 67, "N_OR": 68, "N_XOR": 69, "N_NOT": 70,
    "N_SHL": 71, "N_LSHR": 72, "N_ASHR": 73,
    "N_UDIV": 74, "N_UREM": 75, "N_SDIV": 76, "N_SREM": 77, "N_SMOD": 78,
    "N_ITE": 79, "N_SHLI": 80, "N_LSHRI": 81, "N_SEXT": 82,
    "N_ULTN": 83, "N_ULEN": 84, "N_SLTN": 85, "N_SLEN": 86, "N_EQN": 87,
    "N_UMULNON": 88, "N_ADDCN": 89,
}

# operand classes: 'W' = W slot or 8-word constant, 'N' = N slot or 1-word constant
# (dst class, [src classes for a, b, c])
SHAPES = {
    "END": (None, []), "CHECK": (None, ["N"]), "CHECK_IMP": (None, ["N", "N"]),
    "CHECK_IMPEQ": (None, ["N", "N", "N"]), "CHECK_IMPEQW": (None, ["N", "W", "W"]),
    "CHECK_IMPEQK": (None, ["N", "N", "N"]),   # (N[a] = imm) => (b = c)
    # j = imm - N[a]; j < n => spill word (c & 1023) + j = b, n = (c >> 10 & 31) + 1 (c: a raw field)
    "CHECK_GRID": (None, ["N", "N"]),
    "W_CDINS": ("W", ["W", "W", "W"]),
    "LEAF_W": ("W", []), "LEAF_N": ("N", []),
    "STORE_W": (None, ["W"]), "STORE_N": (None, ["N"]),
    "SPILL_W": (None, ["W"]), "FILL_W": ("W", []), "SPILL_N": (None, ["N"]), "FILL_N": ("N", []),
    "MOV_W": ("W", ["W"]), "MOV_N": ("N", ["N"]),
    "W_ITE": ("W", ["W", "W", "N"]),
    "W_ZEXTN": ("W", ["N"]), "W_SEXTN": ("W", ["N"]), "W_INSN": ("W", ["W", "N"]),
    "W_NOT": ("W", ["W"]), "W_SHLI": ("W", ["W"]), "W_LSHRI": ("W", ["W"]), "W_SEXT": ("W", ["W"]),
    "N_EXTRACTW": ("N", ["W"]),
    "N_NOT": ("N", ["N"]), "N_SHLI": ("N", ["N"]), "N_LSHRI": ("N", ["N"]), "N_SEXT": ("N", ["N"]),
    "N_ITE": ("N", ["N", "N", "N"]),
}
for _n in ("W_ADD", "W_SUB", "W_MUL", "W_AND", "W_OR", "W_XOR", "W_SHL", "W_LSHR", "W_ASHR",
           "W_UDIV", "W_UREM", "W_SDIV", "W_SREM", "W_SMOD"):
    SHAPES[_n] = ("W", ["W", "W"])
for _n in ("N_ULT", "N_ULE", "N_SLT", "N_SLE", "N_EQ", "N_UMULNO", "N_ADDC"):
    SHAPES[_n] = ("N", ["W", "W"])
for _n in ("N_ADD", "N_SUB", "N_MUL", "N_AND", "N_OR", "N_XOR", "N_SHL", "N_LSHR", "N_ASHR",
           "N_UDIV", "N_UREM", "N_SDIV", "N_SREM", "N_SMOD", "N_ULTN", "N_ULEN", "N_SLTN",
           "N_SLEN", "N_EQN", "N_UMULNON", "N_ADDCN"):
    SHAPES[_n] = ("N", ["N", "N"])

FLAG_EARLY_EXIT = 1
FLAG_STOP_AFTER_HIT = 2
FLAG_NO_COUNT = 4      # specialised kernels skip the launch counters (mw_isa.h MW_FLAG_NO_COUNT)


# instruction flags, w0 bits [15:8] (csrc/mw_prog.h)
IMPEQK_LIMIT = 1 << 31   # CHECK_IMPEQK premise constants (bit 31 of the word is free for a chain flag)
FLAG_CHAIN = 1   # W_CDINS: result consumed only by the next W_CDINS's acc (kept in registers)


def encode_dst(cls: str, slot: int = 0) -> int:
    """dst field = the interpreter's write targets (csrc/mw_prog.h): W slot
    [2:0], N low-half slot [7:3], N high-half slot [12:8]; files the op does
    not write get their scratch slot.  cls: "W", "N" or None."""
    w, lo, hi = W_RESERVED, N_RESERVED, N_RESERVED
    if cls == "W":
        w = slot
    elif cls == "N":
        if slot < 32:
            lo = slot
        else:
            hi = slot - 32
    return w | (lo << 3) | (hi << 8)


def decode_dst(dst: int):
    """(W slot, N slot or None) written by an instruction with this dst field."""
    w, lo, hi = dst & 7, (dst >> 3) & 31, (dst >> 8) & 31
    n = lo if lo != N_RESERVED else (32 + hi if hi != N_RESERVED else None)
    return (None if w == W_RESERVED else w), n


def encode(op: str, width: int = 0, dst: int = 0, a: int = 0, b: int = 0, c: int = 0, imm: int = 0,
           flags: int = 0):
    code = OPCODES[op]
    return [(code & 0xFF) | ((flags & 0xFF) << 8) | ((width & 0xFFFF) << 16),
            (dst & 0xFFFF) | ((a & 0xFFFF) << 16),
            (b & 0xFFFF) | ((c & 0xFFFF) << 16),
            imm & 0xFFFFFFFF]


# The threaded-dispatch asm interpreter (csrc/mw_asm_interp.inc, generated by
# tools/gen_asm_interp.py) has a handler for these opcodes and leaf kinds; a
# program using anything else is searched by the compiled interpreter.
ASM_OPCODES = [
    "END", "CHECK", "CHECK_IMP", "CHECK_IMPEQ", "CHECK_IMPEQW", "CHECK_IMPEQK", "LEAF_W", "LEAF_N", "MOV_W", "MOV_N",
    "SPILL_W", "FILL_W", "SPILL_N", "FILL_N",
    "W_ADD", "W_SUB", "W_AND", "W_OR", "W_XOR", "W_NOT", "W_ITE", "W_SHLI", "W_LSHRI", "W_ZEXTN", "W_INSN",
    "W_CDINS", "W_MUL",
    "N_EXTRACTW", "N_ULT", "N_ULE", "N_SLT", "N_SLE", "N_EQ", "N_UMULNO",
    "N_ADD", "N_SUB", "N_AND", "N_OR", "N_XOR", "N_NOT", "N_ITE", "N_SHLI", "N_LSHRI", "N_ULTN", "N_ULEN", "N_EQN",
    "N_MUL", "N_SLTN", "N_SLEN", "N_UMULNON", "N_ADDC", "N_ADDCN",
    "W_UDIV", "W_UREM",
    "STORE_W", "STORE_N",   # trace rows (witness programs, mg_eval_generated)
    "W_SHL", "W_LSHR", "W_ASHR",   # shifts by a per-lane amount (a barrel shifter)
    "CHECK_GRID",   # a congruence grid's row (compiler.py _form_grids)
]
ASM_LEAF_KINDS = [0, 1, 2, 3]
# The asm engines divide bit-serially (256 steps per wide division); a program
# with more wide divisions than this stays on the compiled interpreter and its
# digit-wise udivrem8 (mw_alu.h): C5's 384 divisions among them.
ASM_MAX_DIV = 4
ASM_DIV_OPS = ("W_UDIV", "W_UREM")

# Fused handlers of the asm interpreter: one dispatch runs each sequence, its
# handlers back to back (mythril_amd/asmgen.py gen).  mw_asm_predecode points
# the first instruction of every match at the fused handler, scanning left to
# right, longest sequence first, list order among equal lengths.  Picked by
# tools/opcode_ngrams.py from the committed corpora (profiles/r4n/
# opcode_ngrams.json); W_CDINS (its chains are taken by its own handler) and
# END never join one.
ASM_FUSED_MAX = 4
ASM_FUSED = [
    ("N_SLT", "LEAF_N", "N_ITE", "N_SHLI"),   # a calldata byte behind its bounds guard, shifted into place
    # round 5: the same byte inserted into its word when the leaf has another
    # use, and a grid row after its value's leaf (drawn again there) or fill
    ("N_SLT", "LEAF_N", "N_ITE", "W_INSN"),
    ("LEAF_N", "N_ITE", "W_INSN"),
    ("LEAF_N", "CHECK_GRID"),
    ("FILL_N", "CHECK_GRID"),
    ("N_EQ", "N_EQ", "N_OR", "N_EQ"),
    ("LEAF_W", "LEAF_W", "N_ULE", "CHECK"),
    ("N_OR", "CHECK", "LEAF_W", "N_ULT"),
    ("N_EQ", "N_XOR", "CHECK"),
    ("N_EQ", "CHECK"),
    ("N_SLT", "LEAF_N", "N_ITE"),
    ("N_XOR", "CHECK"),
    ("N_OR", "N_OR"),
    ("LEAF_W", "N_ULE", "CHECK"),
    ("N_EQ", "N_EQ"),
    ("N_OR", "CHECK"),
    ("N_ULT", "N_XOR", "CHECK"),
    ("W_ZEXTN", "N_EQ"),
    ("CHECK", "N_EQ", "CHECK"),
    ("N_XOR", "CHECK", "N_EQ"),
    ("CHECK", "N_EQ"),
    ("LEAF_W", "N_ULE"),
    ("LEAF_W", "N_EQ", "N_EQ", "N_OR"),
    ("LEAF_W", "N_EQ"),
    ("CHECK", "LEAF_W"),
    ("LEAF_N", "N_ITE"),
    ("LEAF_W", "N_ULT"),
]
assert all(2 <= len(t) <= ASM_FUSED_MAX and not {"W_CDINS", "END"} & set(t)
           and set(t) <= set(ASM_OPCODES) for t in ASM_FUSED)


def asm_fused_dispatch(code):
    """[(instruction index, fused sequence index or None)] for the dispatched
    instructions of a program (mw_asm_predecode's match, for tests and tools)"""
    ops = [int(w) & 0xFF for w in list(code)[0::4]]
    seqs = [[OPCODES[n] for n in t] for t in ASM_FUSED]
    out, i = [], 0
    while i < len(ops):
        best, blen = None, 0
        for k, t in enumerate(seqs):
            if len(t) > blen and ops[i:i + len(t)] == t:
                best, blen = k, len(t)
        out.append((i, best))
        i += blen if best is not None else 1
    return out


# narrow (N-class) constants the asm interpreter holds in VGPRs (mw_isa.h MW_ASM_NK)
ASM_NK = 16
# per register layout of the asm interpreter (asmgen.py NKN, mw_asm_interp.inc
# MW_ASM_NK_N / MW_ASM_NK_Q): how many narrow constants fit its constant
# registers, and its LDS budget in words per thread (mw_kernels.hip
# kLdsSpillWordsByLayout: pool rows plus spill words)
ASM_NK_BY_LAYOUT = {"wide": ASM_NK, "narrow": ASM_NK - 2, "quarter": 4}
ASM_LDS_WORDS = {"wide": 80, "narrow": 52, "quarter": 40}


def asm_switches() -> dict:
    """The loader's layout switches (mw_kernels.hip asm_enabled /
    asm_narrow_enabled / asm_quarter_enabled), read from the same variables."""
    import os
    off = lambda k: os.environ.get(k, "1")[:1] == "0"   # noqa: E731
    asm = not off("MYTHRIL_AMD_ASM")
    narrow = asm and not off("MYTHRIL_AMD_ASM_NARROW")
    return {"asm": asm, "narrow": narrow, "quarter": narrow and not off("MYTHRIL_AMD_ASM_QUARTER")}


def asm_narrow_constants(code, consts):
    """The distinct values of N-class constant operands, in first-use order:
    what mw_asm_predecode loads into the asm interpreter's constant VGPRs."""
    out = []
    names = {c: n for n, c in OPCODES.items()}
    w = [int(x) for x in code]
    for i in range(0, len(w), 4):
        shape = SHAPES[names[w[i] & 0xFF]][1]
        fields = (w[i + 1] >> 16, w[i + 2] & 0xFFFF, w[i + 2] >> 16)
        for cls, f in zip(shape, fields):
            if cls == "N" and f & KBIT:
                val = int(consts[f & 0x7FFF])
                if val not in out:
                    out.append(val)
    return out


def asm_eligible(code, leaves, consts=None) -> bool:
    """Host mirror of mw_kernels.hip asm_eligible plus mw_asm_predecode's
    bound: every opcode and leaf kind of the program has an asm handler, at
    most ASM_MAX_DIV wide divisions, and (given the constant pool) at most
    ASM_NK distinct narrow constants.  The LDS fit is decided per launch."""
    ok = {OPCODES[n] for n in ASM_OPCODES}
    ops = [int(w) & 0xFF for w in list(code)[0::4]]
    if any(o not in ok for o in ops):
        return False
    div = {OPCODES[n] for n in ASM_DIV_OPS}
    if sum(o in div for o in ops) > ASM_MAX_DIV:
        return False
    kinds = [int(leaves[i + LEAF_KIND]) for i in range(0, len(leaves), LEAF_WORDS)]
    if not all(k in ASM_LEAF_KINDS for k in kinds):
        return False
    return consts is None or len(asm_narrow_constants(code, consts)) <= ASM_NK


# ---------------------------------------------------------------- executed work
# u32 ops one evaluation of a program executes, priced per instruction of the
# final bytecode with SURVEY §8(d)'s units (compiler.node_cost: L = limbs of
# the operand width).  ops_per_eval prices the lowered DAG instead; the two
# agree where each DAG node is one instruction, and differ where the compiler
# executes less than the DAG states: a congruence grid row (CHECK_GRID, one
# table lookup) stands for n pair checks, a keyed check
# (CHECK_IMPEQK) for its premise compare and its pair.  Data movement (leaf
# draws, spills, fills, moves, trace stores) is not algorithmic work: 0.
def _limbs(width: int) -> int:
    return max(1, (width + 31) // 32)


def _log2c(n: int) -> int:
    k = 0
    while (1 << k) < n:
        k += 1
    return k


def insn_ops(op: str, width: int) -> int:
    """u32 ops one instruction executes (width: the instruction's width field,
    the operand width of compares and checks)."""
    L = _limbs(width)
    if op in ("END", "LEAF_W", "LEAF_N", "STORE_W", "STORE_N", "SPILL_W", "FILL_W", "SPILL_N", "FILL_N",
              "MOV_W", "MOV_N", "CHECK"):
        return 0
    if op == "CHECK_IMP":
        return 2                          # =>
    if op == "CHECK_IMPEQ":
        return 2 + 2                      # narrow = and =>
    if op in ("CHECK_IMPEQW", "CHECK_IMPEQK"):
        return 2 * L + 2 + (2 if op == "CHECK_IMPEQK" else 0)   # = (the premise compare too), =>
    if op == "CHECK_GRID":
        return 1 + 2 + 2 * L + 2          # j = E - key, j < n, table[j] = v, =>
    if op in ("W_ADD", "W_SUB", "W_AND", "W_OR", "W_XOR", "W_NOT", "W_ITE", "W_SHLI", "W_LSHRI", "W_ZEXTN",
              "W_SEXT", "W_SEXTN", "N_ADDC"):
        return L
    if op == "W_MUL":
        return 2 * L * (L + 1)
    if op in ("W_SHL", "W_LSHR", "W_ASHR"):
        return 2 * L + L * max(1, _log2c(L)) if L > 1 else 2
    if op in ("W_UDIV", "W_UREM", "W_SDIV", "W_SREM", "W_SMOD"):
        base = L * (6 * L + 20) + 3 * (2 * L + L * max(1, _log2c(L))) if L > 1 else 20
        return base + (4 * L if op in ("W_SDIV", "W_SREM", "W_SMOD") else 0)
    if op == "W_INSN":
        return 1                          # one narrow part of a concat
    if op == "W_CDINS":
        return 8 + 1 + 1 + 1              # a calldata byte: signed 256-bit bound (L+1), ite, its part of the word
    if op in ("N_ULT", "N_ULE", "N_SLT", "N_SLE"):
        return L + 1
    if op == "N_EQ":
        return 2 * L
    if op == "N_UMULNO":
        return 4 * L * L + L
    if op in ("N_AND", "N_OR", "N_XOR"):
        return 2 if width == 1 else 1     # a Bool connective: one per operand
    if op in ("N_MUL",):
        return 4
    if op in ("N_SHL", "N_LSHR", "N_ASHR", "N_ULTN", "N_ULEN", "N_SLTN", "N_SLEN", "N_EQN"):
        return 2
    if op in ("N_UDIV", "N_UREM"):
        return 20
    if op in ("N_SDIV", "N_SREM", "N_SMOD"):
        return 24
    if op == "N_UMULNON":
        return 5
    return 1                              # N_ADD/SUB/NOT/ITE/SHLI/LSHRI/SEXT/EXTRACTW, N_ADDCN


_OPNAME = {v: k for k, v in OPCODES.items()}


def executed_ops_per_eval(code) -> int:
    """Sum of insn_ops over a program's bytecode (4 words per instruction)."""
    w = [int(x) for x in list(code)[0::4]]
    return sum(insn_ops(_OPNAME[x & 0xFF], x >> 16) for x in w)
