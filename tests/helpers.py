"""Test helpers: host-emulator binding, oracle candidate models, random DAGs."""
from __future__ import annotations

import ctypes
import os
import random
from typing import Dict, List, Optional, Sequence

import numpy as np

from mythril_amd.compiler import Program
from mythril_amd.ir import BOOL, Ctx, Node
from mythril_amd.runtime import MgProgDesc, make_desc
from oracle.philox import leaf_value

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST_EMU = os.path.join(ROOT, "build", "host", "libmw_host_emu.so")
_emu = None


def host_emu():
    global _emu
    if _emu is None:
        if not os.path.exists(HOST_EMU):
            from mythril_amd.build import build_host_emu
            build_host_emu()
        lib = ctypes.CDLL(HOST_EMU)
        lib.mwh_eval.restype = ctypes.c_int
        lib.mwh_eval.argtypes = [ctypes.POINTER(MgProgDesc), ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                 ctypes.c_size_t, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
        lib.mwh_keccak256.restype = ctypes.c_int
        lib.mwh_keccak256.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                      ctypes.c_void_p]
        lib.mg_validate_desc.restype = ctypes.c_int
        lib.mg_validate_desc.argtypes = [ctypes.POINTER(MgProgDesc)]
        lib.mg_last_error.restype = ctypes.c_char_p
        _emu = lib
    return _emu


def emu_eval(p: Program, inputs: Optional[np.ndarray], n: int, seed: int = 0, begin: int = 0, flags: int = 0):
    lib = host_emu()
    d, keep = make_desc(p)
    v = np.zeros(n, dtype=np.uint32)
    t = np.zeros(max(p.n_trace_rows, 1) * n, dtype=np.uint32)
    inp = np.ascontiguousarray(inputs, dtype=np.uint32) if inputs is not None else None
    rc = lib.mwh_eval(ctypes.byref(d), inp.ctypes.data if inp is not None else None, seed, begin, n, flags,
                      v.ctypes.data, t.ctypes.data)
    if rc != 0:
        raise RuntimeError(lib.mg_last_error().decode())
    return v, t.reshape(max(p.n_trace_rows, 1), n)


def oracle_models(p: Program, seed: int, begin: int, n: int) -> List[Dict[str, int]]:
    """Leaf assignments of generated candidates, restated by the oracle (oracle/philox.py)."""
    out = []
    for j in range(n):
        m = {}
        for li, (node, spec) in enumerate(zip(p.leaf_nodes, p.leaf_specs)):
            sd = {"id": spec.key_salt(), "width": spec.width, "shift": spec.shift, "bits": spec.bits, "pool": spec.pool,
                  "hashed": spec.hashed, "stride": spec.stride}
            m[node.name] = leaf_value(sd, seed, begin + j)
        out.append(m)
    return out


WIDTHS = [1, 5, 8, 31, 32, 33, 64, 100, 160, 255, 256]


class RandDag:
    """Random well-typed terms over every op the compiler lowers."""

    def __init__(self, seed: int, widths: Sequence[int] = WIDTHS, nvars: int = 6):
        self.r = random.Random(seed)
        self.ctx = Ctx()
        self.widths = list(widths)
        self.vars = [self.ctx.var(f"v{i}_{w}", w) for i, w in enumerate(self.r.choice(self.widths) for _ in range(nvars))]
        self.bvars = [self.ctx.var(f"b{i}", BOOL) for i in range(2)]

    def special(self, w):
        r = self.r.random()
        m = (1 << w) - 1
        if r < 0.15:
            return 0
        if r < 0.3:
            return m
        if r < 0.4:
            return 1 << (w - 1)
        if r < 0.5:
            return self.r.randrange(0, min(w + 3, m + 1))
        return self.r.getrandbits(w)

    def const(self, w):
        return self.ctx.const(self.special(w), w)

    def leaf(self, w):
        cands = [v for v in self.vars if v.width == w]
        if cands and self.r.random() < 0.7:
            return self.r.choice(cands)
        return self.const(w)

    def bv(self, w: int, depth: int) -> Node:
        c, r = self.ctx, self.r
        if depth <= 0 or r.random() < 0.15:
            return self.leaf(w)
        k = r.random()
        d = depth - 1
        if k < 0.40:
            op = r.choice(["bvadd", "bvsub", "bvmul", "bvand", "bvor", "bvxor", "bvudiv", "bvurem",
                           "bvsdiv", "bvsrem", "bvsmod", "bvshl", "bvlshr", "bvashr", "bvnand", "bvnor",
                           "bvxnor"])
            a = self.bv(w, d)
            b = self.bv(w, d) if op not in ("bvshl", "bvlshr", "bvashr") or r.random() < 0.5 else \
                c.const(r.choice([0, 1, w - 1, w, w + 1, r.randrange(0, w)]) & ((1 << w) - 1), w)
            if op in ("bvadd", "bvmul", "bvand", "bvor", "bvxor") and r.random() < 0.3:
                return c.app(op, a, b, self.bv(w, d))
            return c.app(op, a, b)
        if k < 0.48:
            return c.app(r.choice(["bvneg", "bvnot"]), self.bv(w, d))
        if k < 0.58:
            return c.app("ite", self.boolean(d), self.bv(w, d), self.bv(w, d))
        if k < 0.68 and w > 1:  # concat
            cut = r.randrange(1, w)
            return c.app("concat", self.bv(w - cut, d), self.bv(cut, d))
        if k < 0.78:  # extract from something wider
            big = r.choice([x for x in self.widths if x >= w])
            lo = r.randrange(0, big - w + 1)
            return c.app("extract", self.bv(big, d), params=(lo + w - 1, lo))
        if k < 0.86 and w > 1:
            small = r.choice([x for x in self.widths if x < w] or [1])
            return c.app(r.choice(["zero_extend", "sign_extend"]), self.bv(small, d), params=(w - small,))
        if k < 0.92:
            return c.app(r.choice(["rotate_left", "rotate_right"]), self.bv(w, d), params=(r.randrange(0, 2 * w),))
        if k < 0.95 and w % 2 == 0 and w >= 2:
            return c.app("repeat", self.bv(w // 2, d), params=(2,))
        return c.app("bvcomp", self.bv(w, d), self.bv(w, d)) if w == 1 else self.leaf(w)

    def boolean(self, depth: int) -> Node:
        c, r = self.ctx, self.r
        if depth <= 0 or r.random() < 0.1:
            return r.choice(self.bvars + [c.true(), c.false()])
        k = r.random()
        d = depth - 1
        if k < 0.5:
            w = r.choice(self.widths)
            op = r.choice(["bvult", "bvule", "bvugt", "bvuge", "bvslt", "bvsle", "bvsgt", "bvsge", "=",
                           "distinct", "bvumul_noovfl"])
            return c.app(op, self.bv(w, d), self.bv(w, d))
        if k < 0.8:
            op = r.choice(["and", "or", "xor", "=>", "=", "distinct"])
            return c.app(op, self.boolean(d), self.boolean(d))
        if k < 0.9:
            return c.app("not", self.boolean(d))
        return c.app("ite", self.boolean(d), self.boolean(d), self.boolean(d))


def random_assignments(vars_: Sequence[Node], n: int, rng: random.Random, dag: RandDag) -> List[Dict[str, int]]:
    out = []
    for _ in range(n):
        m = {}
        for v in vars_:
            w = 1 if v.width == BOOL else v.width
            m[v.name] = dag.special(w)
        out.append(m)
    return out


def division_stress_pairs(n: int, seed: int, w: int = 256):
    """(x, y) pairs shaped to reach Knuth D's rare corrections: divisors with
    structured top limbs over all-ones / random low limbs, dividends y*q + r with
    q near the digit base.  Most sets of a few dozen include quotient estimates
    that are one too large (add-back) and equal top words (qhat = B-1)."""
    rng = random.Random(seed)
    B = 1 << 32
    m = (1 << w) - 1
    out = []
    while len(out) < n:
        nb = rng.randint(min(33, w), w)
        top = rng.choice([B - 1, 1 << 31, (1 << 31) | 1, rng.getrandbits(32) | (1 << 31)])
        lo_bits = max(nb - 32, 0)
        y = (top << lo_bits) | (((1 << lo_bits) - 1) if rng.random() < 0.5 else rng.getrandbits(lo_bits) if lo_bits else 0)
        y &= m
        if y == 0:
            continue
        q = rng.choice([B - 1, B - 2, B, rng.getrandbits(32), (1 << 64) - 1])
        x = (y * q + rng.choice([0, y - 1, rng.getrandbits(max(1, nb - 1))])) & m
        out.append((x, y))
    return out


def division_check_programs(npairs: int = 256, seed: int = 11):
    """Programs asserting op(a, b) == e for the five divisions, where candidate i
    draws (a, b, e) = pair i and its oracle result from bit-field pools (same
    digit): every verdict over candidates [0, npairs) must be 1."""
    from mythril_amd.compiler import LeafSpec, compile_program
    from oracle import bvsem
    pairs = division_stress_pairs(npairs, seed)
    k = (npairs - 1).bit_length()
    progs = []
    for op in ("bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod"):
        ctx = Ctx()
        a, b, e = ctx.var("a", 256), ctx.var("b", 256), ctx.var("e", 256)
        exp = [getattr(bvsem, op)(256, x, y) for x, y in pairs]
        specs = {nm: LeafSpec(nm, 256, pool=list(vals), shift=0, bits=k)
                 for nm, vals in (("a", [x for x, _ in pairs]), ("b", [y for _, y in pairs]), ("e", exp))}
        progs.append(compile_program([ctx.app("=", ctx.app(op, a, b), e)], leaf_specs=specs))
    return progs


def mul_stress_pairs(n: int, seed: int = 13):
    """256-bit operand pairs for the column multiply (mw_jit.h mul8_cols):
    limbs from the carry-heavy set (all ones, 2^32 - 2, the top bit, 0, 1)
    mixed with random limbs, whole-word edge values, and random pairs."""
    rng = random.Random(seed)
    M = (1 << 256) - 1
    edge = [0xFFFFFFFF, 0xFFFFFFFE, 0x80000000, 0, 1, 0x7FFFFFFF]

    def word(mode):
        if mode == 0:
            return rng.getrandbits(256)
        if mode == 1:
            return M - rng.getrandbits(rng.choice([0, 1, 8, 32, 64, 200]))
        return sum((rng.choice(edge) if rng.random() < 0.7 else rng.getrandbits(32)) << (32 * k) for k in range(8))
    out = [(M, M), (M, 1), (1 << 255, M), (M, (1 << 32) - 1)]
    while len(out) < n:
        out.append((word(rng.randrange(3)), word(rng.randrange(3))))
    return out[:n]


def mul_check_programs(npairs: int = 4096, seed: int = 13):
    """One program asserting bvmul(a, b) == e and bvmul(b, a) == e, where
    candidate i draws (a, b, e) = pair i of mul_stress_pairs and its oracle
    product from bit-field pools: every verdict over [0, npairs) must be 1."""
    from mythril_amd.compiler import LeafSpec, compile_program
    from oracle import bvsem
    pairs = mul_stress_pairs(npairs, seed)
    k = (npairs - 1).bit_length()
    ctx = Ctx()
    a, b, e = ctx.var("a", 256), ctx.var("b", 256), ctx.var("e", 256)
    exp = [bvsem.bvmul(256, x, y) for x, y in pairs]
    specs = {nm: LeafSpec(nm, 256, pool=list(vals), shift=0, bits=k)
             for nm, vals in (("a", [x for x, _ in pairs]), ("b", [y for _, y in pairs]), ("e", exp))}
    conj = [ctx.app("=", ctx.app("bvmul", a, b), e), ctx.app("=", ctx.app("bvmul", b, a), e)]
    return [compile_program(conj, leaf_specs=specs)]


def full_width_division_models(seed: int, n: int) -> List[Dict[str, int]]:
    """Operand pairs whose divisor has a nonzero top limb (y >= 2^224), with the
    quotient-estimate edge cases of mw_alu.h udivrem8_full: digits near 2^32-1,
    exact multiples and their neighbours, x < y, x = y, 64-bit heads that round."""
    rng = random.Random(seed)
    M = (1 << 256) - 1
    ys = [1 << 224, (1 << 224) + 1, M, 1 << 255, (1 << 255) - 1, ((1 << 32) - 1) << 224,
          (1 << 224) | ((1 << 192) - 1), (1 << 224) + (1 << 192), ((1 << 53) + 1) << 203]
    out = []
    while len(out) < n:
        y = rng.choice(ys) if rng.random() < 0.5 else (rng.getrandbits(256) | (1 << (224 + rng.randrange(32))))
        k = rng.choice([0, 1, 2, 3, (1 << 31), (1 << 32) - 1, (1 << 32) - 2, rng.getrandbits(32)])
        d = rng.choice([0, 1, -1, y - 1, rng.getrandbits(200)])
        x = k * y + d
        if rng.random() < 0.1:
            x = rng.choice([0, 1, M, y - 1, y, y + 1, M - 1])
        out.append({"a": x & M, "b": y})
    return out


def short_division_models(seed: int, n: int) -> List[Dict[str, int]]:
    """Operand pairs with one-limb divisors (0 < y < 2^32) in every model: the
    short-division path of mw_alu.h (udivrem8_short), normalisation shifts 0..31
    and the 2-by-1 corrections."""
    rng = random.Random(seed)
    M = (1 << 256) - 1
    ys = [1, 2, 3, 7, (1 << 31) - 1, 1 << 31, (1 << 31) + 1, (1 << 32) - 1, (1 << 32) - 2, 0x10001]
    out = []
    while len(out) < n:
        y = rng.choice(ys) if rng.random() < 0.5 else rng.randrange(1, 1 << rng.randint(1, 32))
        x = rng.choice([rng.getrandbits(256), M, 0, y - 1, y, rng.getrandbits(256) // y * y,
                        rng.getrandbits(256) // y * y - 1, rng.getrandbits(40)])
        out.append({"a": x & M, "b": y})
    return out


CONSTANT_DIVISORS = [0, 1, 3, 1 << 31, (1 << 31) + 1, (1 << 32) - 1, 1 << 32, 1 << 224, (1 << 224) + 1,
                     1 << 255, (1 << 256) - 1, 0x10001 << 128]


def constant_divisor_programs(npairs: int = 256, seed: int = 12):
    """One program per constant divisor K asserting op(a, K) == e_op for the five
    divisions, with a and the oracle's results e_op drawn from bit-field pools
    (same digit): every verdict over candidates [0, npairs) must be 1.  A
    specialised kernel sees K as literals, so LLVM constant-folds the divisor's
    normalisation and reciprocal (d = 2^31 once folded an out-of-range
    double -> u32 conversion to poison)."""
    from mythril_amd.compiler import LeafSpec, compile_program
    from oracle import bvsem
    rng = random.Random(seed)
    M = (1 << 256) - 1
    k = (npairs - 1).bit_length()
    ops = ("bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod")
    progs = []
    for K in CONSTANT_DIVISORS:
        xs = [0, 1, M, M - 1, 1 << 255, (K - 1) & M, K, (K + 1) & M]
        while len(xs) < npairs:
            xs.append(rng.getrandbits(256) if rng.random() < 0.7 else (rng.getrandbits(40) * K + rng.choice([0, 1, K - 1])) & M)
        ctx = Ctx()
        a = ctx.var("a", 256)
        specs = {"a": LeafSpec("a", 256, pool=xs, shift=0, bits=k)}
        conj = []
        for op in ops:
            e = ctx.var("e_" + op, 256)
            specs["e_" + op] = LeafSpec("e_" + op, 256, pool=[getattr(bvsem, op)(256, x, K) for x in xs], shift=0, bits=k)
            conj.append(ctx.app("=", ctx.app(op, a, ctx.const(K, 256)), e))
        progs.append(compile_program(conj, leaf_specs=specs))
    return progs
