"""Python mirror of ``csrc/mw_isa.h`` (kept in sync by tests/test_isa_sync.py)."""
from __future__ import annotations

NW = 8           # W file slots (8 x u32 limbs each)
NN = 64          # N file slots (1 x u32 each)
W_RESERVED = NW - 1   # interpreter write-back scratch slots, never allocated (mw_isa.h)
N_RESERVED = 31       # N slots 31 and 63
KBIT = 0x8000
LEAF_WORDS = 8
POOL_ENTRY_WORDS = 9
MAX_WIDTH = 256
NARROW_MAX = 32

LEAF_WIDTH, LEAF_KIND, LEAF_ID, LEAF_SHIFT, LEAF_BITS, LEAF_POOL, LEAF_INROW = range(7)

OPCODES = {
    "END": 0, "CHECK": 1, "LEAF_W": 2, "LEAF_N": 3, "STORE_W": 4, "STORE_N": 5,
    "SPILL_W": 6, "FILL_W": 7, "MOV_W": 8, "MOV_N": 9, "SPILL_N": 10, "FILL_N": 11, "CHECK_IMP": 12,
    "CHECK_IMPEQ": 13, "CHECK_IMPEQW": 14,
    "W_ADD": 16, "W_SUB": 17, "W_MUL": 18, "W_AND": 19, "W_OR": 20, "W_XOR": 21, "W_NOT": 22,
    "W_SHL": 23, "W_LSHR": 24, "W_ASHR": 25,
    "W_UDIV": 26, "W_UREM": 27, "W_SDIV": 28, "W_SREM": 29, "W_SMOD": 30,
    "W_ITE": 31, "W_SHLI": 32, "W_LSHRI": 33, "W_ZEXTN": 34, "W_SEXT": 35, "W_SEXTN": 36,
    "W_INSN": 37, "W_CDINS": 38,
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


# instruction flags, w0 bits [15:8] (csrc/mw_prog.h)
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
