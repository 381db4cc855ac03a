"""Round-5 congruence rewrites in lower.py, checked by evaluation: the
lowered set with each rewrite is the same Boolean function of the leaves as
the lowered set without it (oracle.dag_eval on random assignments, with the
values the rewrites depend on planted often enough to make both outcomes
occur):

* pinned leaves (lower._pins): a read whose value leaf a top-level conjunct
  fixes is compared as that constant in its pairs;
* shared arguments: premise parts over an argument both reads share are dropped;
* keyed premises (lower._Rewriter.keyed) over nested constant offsets
  (lower._offset folds off + 4 + k)."""
import random

from mythril_amd import lower
from mythril_amd.ir import Ctx
from oracle.dag_eval import eval_nodes


def _leaves(nodes):
    return {n.name: n.width for n in nodes if n.op == "var"}


def _holds(low, model):
    vals = eval_nodes(low.conjuncts, model)
    return all(vals[c.id] for c in low.conjuncts)


def _compare(c, conj, monkeypatch, disable, rng, n=400, plant=None):
    with_rw = lower.lower_constraints(conj, c)
    with monkeypatch.context() as m:
        disable(m)
        without = lower.lower_constraints(conj, c)
    assert [x.id for x in with_rw.conjuncts] != [x.id for x in without.conjuncts], "the rewrite did nothing"
    names = {**_leaves(with_rw.nodes), **_leaves(without.nodes)}
    seen = set()
    for _ in range(n):
        model = {k: rng.getrandbits(w) for k, w in names.items()}
        if plant:
            plant(model, rng)
        a, b = _holds(with_rw, model), _holds(without, model)
        assert a == b, model
        seen.add(a)
    assert seen == {True, False}, seen


def test_pinned_leaves(monkeypatch):
    """Power(256, k) = 256^k for k < 4 and Power(256, x) > 0: the pairs
    compare Power(256, x)'s leaf with the constants."""
    c = Ctx()
    x = c.var("x", 256)
    pw = [c.apply("Power", 256, c.const(256, 256), c.const(k, 256)) for k in range(4)]
    px = c.apply("Power", 256, c.const(256, 256), x)
    conj = [c.app("=", p, c.const(256 ** k, 256)) for k, p in enumerate(pw)]
    conj += [c.app("bvult", x, c.const(6, 256)), c.app("bvugt", px, c.const(0, 256))]
    low = lower.lower_constraints(conj, c)
    cong = low.conjuncts[-low.congruence:]
    assert any(n.op == "const" and n.val == 256 ** 2 for cj in cong for n in [cj] + list(cj.args[1].args)
               if cj.op == "=>"), "no pinned constant in the pairs"

    def plant(model, rng):
        model["x"] = rng.randrange(6)
        for name in list(model):
            if name.startswith("Power@100,") and rng.random() < 0.9:      # a pinned cell: its constant
                model[name] = 256 ** int(name.split(",")[1], 16)
            elif name.startswith("Power@s") and rng.random() < 0.7:       # the symbolic cell: x's power
                model[name] = 256 ** model["x"] if model["x"] < 4 else rng.getrandbits(256)

    _compare(c, conj, monkeypatch, lambda m: m.setattr(lower, "_pins", lambda out, ack: {}),
             random.Random(1), plant=plant)


def test_shared_argument_drops_from_premise(monkeypatch):
    """f(256, k) against f(256, x): the premise is x = k alone."""
    c = Ctx()
    x = c.var("x", 256)
    fs = [c.apply("F", 8, c.const(256, 256), c.const(k, 256)) for k in range(3)]
    fx = c.apply("F", 8, c.const(256, 256), x)
    conj = [c.app("bvult", x, c.const(4, 256)), c.app("bvult", fx, c.const(200, 8))]
    conj += [c.app("bvuge", f, c.const(0, 8)) for f in fs] + [c.app("not", c.app("=", fs[0], fs[1]))]
    low = lower.lower_constraints(conj, c)
    prem = [cj.args[0] for cj in low.conjuncts[-low.congruence:] if cj.op == "=>"]
    assert prem and all(p.op != "and" for p in prem)

    def plant(model, rng):
        model["x"] = rng.randrange(4)
        for name in list(model):
            if name.startswith("F"):
                model[name] = rng.randrange(4)

    def pair_with_shared(self, t, u):
        cc = self.ctx
        if all(a.op == "const" for a in t.args) and all(a.op == "const" for a in u.args):
            return None
        if any(lower._never_equal(p, q) for p, q in zip(t.args, u.args)):
            return None
        same = [self.eq(*lower._fold_offsets(cc, p, q)) for p, q in zip(t.args, u.args)]
        prem = cc.app("and", *same) if len(same) > 1 else same[0]
        return cc.app("=>", prem, self.eq(self._value(t), self._value(u)))

    _compare(c, conj, monkeypatch, lambda m: m.setattr(lower._Rewriter, "_pair", pair_with_shared),
             random.Random(2), plant=plant)


def test_keyed_premises_over_nested_offsets(monkeypatch):
    """cd[(off + 4) + k] against cd[K]: one key for the word, premises
    key = K - 4 - k + 2^16, equal to the unkeyed set (KEY_MIN out of reach)
    on offsets that put the word over, beside and past the concrete cells,
    and at wrap-around."""
    c = Ctx()
    cd = c.array("cd", 256, 8)
    off = c.var("off", 256)
    base = c.app("bvadd", off, c.const(4, 256))
    sym = [c.app("select", cd, c.app("bvadd", base, c.const(k, 256)) if k else base) for k in range(12)]
    con = [c.app("select", cd, c.const(k, 256)) for k in range(16)]
    conj = [c.app("bvule", s, c.const(250, 8)) for s in sym] + [c.app("bvuge", k, c.const(1, 8)) for k in con]
    low = lower.lower_constraints(conj, c)
    keys = {cj.args[0].args[0].id for cj in low.conjuncts[-low.congruence:]
            if cj.op == "=>" and cj.args[0].op == "=" and cj.args[0].args[0].op == "ite"}
    assert len(keys) == 1, keys

    def plant(model, rng):
        model["off"] = rng.choice([0, 1, 5, 11, 20, (1 << 256) - 4, (1 << 256) - 9, rng.getrandbits(256)])
        for name in list(model):
            if name.startswith("cd"):
                model[name] = rng.choice([1, 2, 3])

    _compare(c, conj, monkeypatch, lambda m: m.setattr(lower, "KEY_MIN", 1 << 30), random.Random(3), plant=plant)
