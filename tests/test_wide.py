"""Wide (> 256-bit) bitvector terms: legalisation into 256-bit chunks (lower.py).

Mythril builds wider terms in two places: BVAddNoOverflow's 257-bit add
(mythril/laser/smt/bitvec_helper.py:196-208 -> z3 Z3_mk_bvadd_no_overflow:
``extract(256, 256, zext1(a) + zext1(b)) == 0``; SWC-101 at
mythril/analysis/module/modules/integer.py:143) and 512-bit and wider keccak
inputs (mythril/laser/ethereum/instructions.py:1016-1030).  The lowered
programs run on the host build of the interpreter here (tests/test_gpu_wide.py
runs them on gfx950) and must agree with the oracle's big-int evaluation of
the ORIGINAL wide formula.
"""
import random

import pytest

from mythril_amd import isa
from mythril_amd.compiler import Unsupported, compile_program
from mythril_amd.engine import prepare
from mythril_amd.ir import BOOL, Ctx
from mythril_amd.lower import MAXW
from mythril_amd.runtime import pack_inputs
from oracle.dag_eval import eval_nodes
from tests.helpers import emu_eval

WIDE_WIDTHS = [1, 8, 64, 200, 256, 257, 300, 512]


def split_model(m, widths):
    """Add the 256-bit chunk leaves (name#k, LSB first) of every wide variable."""
    out = dict(m)
    for name, v in m.items():
        w = widths.get(name, 0)
        if w > MAXW:
            for k, lo in enumerate(range(0, w, MAXW)):
                out[f"{name}#{k}"] = (v >> lo) & ((1 << min(MAXW, w - lo)) - 1)
    return out


def host_run(p, inputs, n):
    return emu_eval(p, inputs, n)[0]


RUN = {"eval": host_run}   # tests/test_gpu_wide.py swaps in the device


def check(conj, models, ctx, want_opcode=None):
    q = prepare(conj, ctx, use_pools=False)
    p = q.program
    widths = {n.name: n.width for n in ctx.nodes if n.op == "var"}
    rows = [split_model(m, widths) for m in models]
    got = RUN["eval"](p, pack_inputs(p, rows), len(rows))
    for j, m in enumerate(models):
        vals = eval_nodes(conj, m)
        want = int(all(vals[c.id] for c in conj))
        assert int(got[j]) == want, (j, m)
    if want_opcode:
        ops = {int(w) & 0xFF for w in p.code.reshape(-1, 4)[:, 0]}
        assert isa.OPCODES[want_opcode] in ops
    return p


def boundary(w, r):
    m = (1 << w) - 1
    return r.choice([0, 1, m, m - 1, 1 << (w - 1), (1 << (w - 1)) - 1, r.getrandbits(w), r.getrandbits(w)])


def test_bvadd_no_overflow_257_bit_pattern():
    """Not(BVAddNoOverflow(a, b, False)), the SWC-101 add check, reaches the
    device as one carry-out instruction (N_ADDC)."""
    c = Ctx()
    a, b = c.var("a", 256), c.var("b", 256)
    s = c.app("bvadd", c.app("zero_extend", a, params=(1,)), c.app("zero_extend", b, params=(1,)))
    noovf = c.app("=", c.app("extract", s, params=(256, 256)), c.const(0, 1))
    conj = [c.app("not", noovf)]
    r = random.Random(7)
    M = (1 << 256) - 1
    models = [{"a": M, "b": 1}, {"a": M, "b": 0}, {"a": 1 << 255, "b": 1 << 255}, {"a": (1 << 255) - 1, "b": 1 << 255},
              {"a": 0, "b": 0}] + [{"a": boundary(256, r), "b": boundary(256, r)} for _ in range(300)]
    p = check(conj, models, c, "N_ADDC")
    assert p.n_insn < 12   # leaves, the carry, the check: no 257-bit arithmetic left


@pytest.mark.parametrize("w", [257, 300, 512, 1024])
def test_wide_add_sub_compare(w):
    c = Ctx()
    x, y = c.var("x", w), c.var("y", w)
    r = random.Random(w)
    shapes = [
        [c.app("bvult", c.app("bvadd", x, y), x)],                      # wrapped add
        [c.app("=", c.app("bvsub", x, y), c.const(5, w))],
        [c.app("bvsle", c.app("bvneg", x), y)],
        [c.app("bvuge", c.app("bvadd", x, y, c.const(3, w)), c.app("bvxor", x, y))],
        [c.app("distinct", c.app("bvnot", x), c.app("bvor", x, y))],
        [c.app("bvsgt", c.app("ite", c.app("bvult", x, y), x, y), c.const(1 << (w - 1), w))],
    ]
    models = [{"x": boundary(w, r), "y": boundary(w, r)} for _ in range(160)]
    models += [{"x": v, "y": (v - 5) % (1 << w)} for v in (0, 3, 5, (1 << w) - 1)]
    for conj in shapes:
        check(conj, models, c)


@pytest.mark.parametrize("w", [257, 512])
def test_wide_structure_and_constant_shifts(w):
    c = Ctx()
    x = c.var("x", w)
    lo = c.var("lo", 200)
    r = random.Random(3 * w)
    terms = [
        c.app("bvshl", x, c.const(37, w)), c.app("bvlshr", x, c.const(260, w)),
        c.app("bvashr", x, c.const(5, w)), c.app("bvashr", x, c.const(w + 9, w)),
        c.app("rotate_left", x, params=(100,)), c.app("rotate_right", x, params=(3,)),
        c.app("concat", c.app("extract", x, params=(w - 1, 200)), lo),
        c.app("bvadd", c.app("sign_extend", lo, params=(w - 200,)), x),
        c.app("repeat", c.app("extract", x, params=(w // 2 - 1, 0)), params=(2,)) if w % 2 == 0 else x,
    ]
    k = c.const(r.getrandbits(w), w)
    conj_sets = [[c.app("bvule", t, k)] for t in terms] + \
                [[c.app("=", c.app("extract", t, params=(w - 2, 250)), c.app("extract", x, params=(w - 2, 250)))]
                 for t in terms]
    models = [{"x": boundary(w, r), "lo": boundary(200, r)} for _ in range(120)]
    for conj in conj_sets:
        check(conj, models, c)


class WideDag:
    """Random terms over the legalised wide vocabulary (no wide mul/div/variable shift)."""

    def __init__(self, seed):
        self.r = random.Random(seed)
        self.c = Ctx()
        self.vars = {w: [self.c.var(f"v{w}_{i}", w) for i in range(2)] for w in WIDE_WIDTHS}

    def bv(self, w, d):
        c, r = self.c, self.r
        if d <= 0 or r.random() < 0.2:
            return r.choice(self.vars[w]) if r.random() < 0.8 else c.const(boundary(w, r), w)
        k = r.random()
        if k < 0.35:
            op = r.choice(["bvadd", "bvsub", "bvand", "bvor", "bvxor"])
            return c.app(op, self.bv(w, d - 1), self.bv(w, d - 1))
        if k < 0.45:
            return c.app(r.choice(["bvneg", "bvnot"]), self.bv(w, d - 1))
        if k < 0.55:
            return c.app("ite", self.boolean(d - 1), self.bv(w, d - 1), self.bv(w, d - 1))
        if k < 0.65 and w > 1:
            smaller = [x for x in WIDE_WIDTHS if x < w]
            cut = r.choice(smaller)
            rest = w - cut
            hi = self.bv(rest, d - 1) if rest in self.vars else c.app("extract", self.bv(512, d - 1),
                                                                         params=(rest - 1, 0))
            return c.app("concat", hi, self.bv(cut, d - 1))
        if k < 0.75:
            big = r.choice([x for x in WIDE_WIDTHS if x >= w])
            lo = r.randrange(0, big - w + 1)
            return c.app("extract", self.bv(big, d - 1), params=(lo + w - 1, lo))
        if k < 0.85 and w > 1:
            small = r.choice([x for x in WIDE_WIDTHS if x < w])
            return c.app(r.choice(["zero_extend", "sign_extend"]), self.bv(small, d - 1), params=(w - small,))
        if k < 0.93:
            op = r.choice(["bvshl", "bvlshr", "bvashr"])
            return c.app(op, self.bv(w, d - 1), c.const(r.choice([0, 1, 31, 32, 255, 256, 257, w - 1, w]) % (1 << w), w))
        return c.app(r.choice(["rotate_left", "rotate_right"]), self.bv(w, d - 1), params=(r.randrange(0, 2 * w),))

    def boolean(self, d):
        c, r = self.c, self.r
        w = r.choice(WIDE_WIDTHS)
        op = r.choice(["bvult", "bvule", "bvugt", "bvuge", "bvslt", "bvsle", "bvsgt", "bvsge", "=", "distinct"])
        return c.app(op, self.bv(w, d), self.bv(w, d))


@pytest.mark.parametrize("seed", range(16))
def test_random_wide_dags(seed):
    g = WideDag(1000 + seed)
    conj = [g.boolean(3) for _ in range(3)]
    models = []
    for _ in range(48):
        models.append({v.name: boundary(w, g.r) for w, vs in g.vars.items() for v in vs})
    check(conj, models, g.c)


@pytest.mark.parametrize("op", ["bvmul", "bvudiv", "bvurem", "bvsdiv", "bvshl-var"])
def test_wide_nonlinear_fails_closed(op):
    c = Ctx()
    x, y = c.var("x", 512), c.var("y", 512)
    t = c.app("bvshl", x, y) if op == "bvshl-var" else c.app(op, x, y)
    with pytest.raises(Unsupported):
        prepare([c.app("bvult", t, c.const(9, 512))], c, use_pools=False)
