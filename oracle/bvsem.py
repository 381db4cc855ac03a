"""ORACLE (test infrastructure only): SMT-LIB 2.6 bitvector/Bool semantics.

Pure-Python big-int restatement of the term semantics z3 gives the operators
Mythril builds constraints from.  Values are non-negative Python ints below
``2**w``; Bools are ``0``/``1``.

Reference call sites (the op vocabulary):
  bitvec.py:126-166   ``+ - * /`` -> bvadd, bvsub, bvmul, **bvsdiv** (``/`` is signed)
  bitvec.py:168-199   ``& | ^``   -> bvand, bvor, bvxor
  bitvec.py:201-243   ``< > <= >=`` -> **signed** bvslt/bvsgt/bvsle/bvsge
  bitvec.py:79-85,246-279 ``==``/``!=`` zero-pad the narrower side (sha3 512-bit values)
  bitvec.py:295-309   ``<<`` -> bvshl, ``>>`` -> **bvashr**
  bitvec_helper.py:30-31  LShR -> bvlshr;  :44-68 If -> ite
  bitvec_helper.py:71-108 UGT/ULT; UGE = Or(UGT, ==) :81-88; ULE = Or(ULT, ==) :101-108
  bitvec_helper.py:121-150 Concat / Extract;  :153-180 URem / SRem / UDiv;  :183-193 Sum
  bitvec_helper.py:196-242 BVAddNoOverflow / BVMulNoOverflow / BVSubNoUnderflow
  bool.py:340-376     And / Xor / Or / Not
Division-by-zero and over-wide shift behaviour follows SMT-LIB 2.6 (z3's
default ``hi_div0=true``): pinned by ``tests/instructions/shl_test.py:30-32``
and ``sar_test.py:32,79-87`` (shift >= 256) — see tests/golden/eip145.json.
"""
from __future__ import annotations

from typing import Sequence


def mask(w: int) -> int:
    return (1 << w) - 1


def to_signed(x: int, w: int) -> int:
    return x - (1 << w) if (x >> (w - 1)) & 1 else x


def from_signed(x: int, w: int) -> int:
    return x & mask(w)


# --- arithmetic ---------------------------------------------------------------
def bvadd(w, *xs):
    s = 0
    for x in xs:
        s += x
    return s & mask(w)


def bvsub(w, a, b):
    return (a - b) & mask(w)


def bvneg(w, a):
    return (-a) & mask(w)


def bvmul(w, *xs):
    p = 1
    for x in xs:
        p = (p * x) & mask(w)
    return p


def bvudiv(w, a, b):
    # SMT-LIB: (bvudiv s #b0..0) = #b1..1
    return mask(w) if b == 0 else a // b


def bvurem(w, a, b):
    # SMT-LIB: (bvurem s #b0..0) = s
    return a if b == 0 else a % b


def _msb(x, w):
    return (x >> (w - 1)) & 1


def bvsdiv(w, s, t):
    # SMT-LIB 2.6 FixedSizeBitVectors definition of bvsdiv
    ms, mt = _msb(s, w), _msb(t, w)
    if not ms and not mt:
        return bvudiv(w, s, t)
    if ms and not mt:
        return bvneg(w, bvudiv(w, bvneg(w, s), t))
    if not ms and mt:
        return bvneg(w, bvudiv(w, s, bvneg(w, t)))
    return bvudiv(w, bvneg(w, s), bvneg(w, t))


def bvsrem(w, s, t):
    ms, mt = _msb(s, w), _msb(t, w)
    if not ms and not mt:
        return bvurem(w, s, t)
    if ms and not mt:
        return bvneg(w, bvurem(w, bvneg(w, s), t))
    if not ms and mt:
        return bvurem(w, s, bvneg(w, t))
    return bvneg(w, bvurem(w, bvneg(w, s), bvneg(w, t)))


def bvsmod(w, s, t):
    ms, mt = _msb(s, w), _msb(t, w)
    abs_s = s if not ms else bvneg(w, s)
    abs_t = t if not mt else bvneg(w, t)
    u = bvurem(w, abs_s, abs_t)
    if u == 0:
        return u
    if not ms and not mt:
        return u
    if ms and not mt:
        return bvadd(w, bvneg(w, u), t)
    if not ms and mt:
        return bvadd(w, u, t)
    return bvneg(w, u)


# --- bitwise ------------------------------------------------------------------
def bvand(w, *xs):
    r = mask(w)
    for x in xs:
        r &= x
    return r


def bvor(w, *xs):
    r = 0
    for x in xs:
        r |= x
    return r


def bvxor(w, *xs):
    r = 0
    for x in xs:
        r ^= x
    return r


def bvnot(w, a):
    return a ^ mask(w)


def bvnand(w, a, b):
    return bvnot(w, a & b)


def bvnor(w, a, b):
    return bvnot(w, a | b)


def bvxnor(w, a, b):
    return bvnot(w, a ^ b)


# --- shifts -------------------------------------------------------------------
def bvshl(w, a, b):
    return 0 if b >= w else (a << b) & mask(w)


def bvlshr(w, a, b):
    return 0 if b >= w else a >> b


def bvashr(w, a, b):
    sa = to_signed(a, w)
    if b >= w:
        return mask(w) if sa < 0 else 0
    return from_signed(sa >> b, w)


def rotate_left(w, n, a):
    n %= w
    return ((a << n) | (a >> (w - n))) & mask(w) if n else a


def rotate_right(w, n, a):
    n %= w
    return ((a >> n) | (a << (w - n))) & mask(w) if n else a


# --- structural ---------------------------------------------------------------
def concat(widths: Sequence[int], xs: Sequence[int]) -> int:
    # first argument is the most significant
    r = 0
    for wi, x in zip(widths, xs):
        r = (r << wi) | x
    return r


def extract(hi, lo, a):
    return (a >> lo) & mask(hi - lo + 1)


def zero_extend(w_in, n, a):
    return a


def sign_extend(w_in, n, a):
    return from_signed(to_signed(a, w_in), w_in + n)


def repeat(w_in, n, a):
    r = 0
    for _ in range(n):
        r = (r << w_in) | a
    return r


# --- predicates (result 0/1) --------------------------------------------------
def bvult(w, a, b):
    return int(a < b)


def bvule(w, a, b):
    return int(a <= b)


def bvugt(w, a, b):
    return int(a > b)


def bvuge(w, a, b):
    return int(a >= b)


def bvslt(w, a, b):
    return int(to_signed(a, w) < to_signed(b, w))


def bvsle(w, a, b):
    return int(to_signed(a, w) <= to_signed(b, w))


def bvsgt(w, a, b):
    return int(to_signed(a, w) > to_signed(b, w))


def bvsge(w, a, b):
    return int(to_signed(a, w) >= to_signed(b, w))


def bvumul_noovfl(w, a, b):
    # z3 Z3_mk_bvmul_no_overflow(signed=False): full product fits in w bits
    return int(a * b < (1 << w))


def bvsmul_noovfl(w, a, b):
    return int(to_signed(a, w) * to_signed(b, w) <= (1 << (w - 1)) - 1)


def bvsmul_noudfl(w, a, b):
    return int(to_signed(a, w) * to_signed(b, w) >= -(1 << (w - 1)))


def bvaddc(w, a, b):
    # internal (mythril_amd/lower.py wide-arithmetic legalisation): carry out of the
    # w-bit addition a + b, i.e. bit w of the (w+1)-bit sum of the zero-extended operands
    return int(a + b >= (1 << w))


# Table used by dag_eval: op -> callable(width_of_first_arg, *values)
BINARY_PRED = {
    "bvaddc": bvaddc,
    "bvult": bvult, "bvule": bvule, "bvugt": bvugt, "bvuge": bvuge,
    "bvslt": bvslt, "bvsle": bvsle, "bvsgt": bvsgt, "bvsge": bvsge,
    "bvumul_noovfl": bvumul_noovfl, "bvsmul_noovfl": bvsmul_noovfl,
    "bvsmul_noudfl": bvsmul_noudfl,
}

NARY_BV = {"bvadd": bvadd, "bvmul": bvmul, "bvand": bvand, "bvor": bvor, "bvxor": bvxor}

BINARY_BV = {
    "bvsub": bvsub, "bvudiv": bvudiv, "bvurem": bvurem, "bvsdiv": bvsdiv,
    "bvsrem": bvsrem, "bvsmod": bvsmod, "bvshl": bvshl, "bvlshr": bvlshr,
    "bvashr": bvashr, "bvnand": bvnand, "bvnor": bvnor, "bvxnor": bvxnor,
}

UNARY_BV = {"bvneg": bvneg, "bvnot": bvnot}
