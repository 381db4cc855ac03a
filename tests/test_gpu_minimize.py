"""Minimize assistance (analysis/solver.py:216-256) on the
device: for small-domain queries the device witness gives
the hint obj_0 <= witness(obj_0).  Checked here: the witness satisfies the
constraints (oracle), so the bound holds for it, and the brute-force optimum
of obj_0 is <= the bound, so z3's optimum is preserved.  The share of obj_0's
domain the hint removes is printed (what Optimize no longer has to refute):
with the device descent (up to 8 more searches below the best value) the
bound is the optimum itself in most cases.  Still opt-in
(MYTHRIL_AMD_MINIMIZE_HINTS=1)."""
import random
import types

import numpy as np
import pytest

from mythril_amd import model as dropin
from mythril_amd import z3bridge
from mythril_amd.engine import WitnessEngine
from oracle.dag_eval import eval_nodes
from tests.test_dropin import CTX, FakeRaw, fb, mythril  # noqa: F401 (fixture)

pytestmark = pytest.mark.gpu

XW, YW = 12, 8


@pytest.fixture(scope="module")
def device():
    from mythril_amd.runtime import Device
    d = Device(0)
    yield d
    d.close()


def _queries():
    """(constraints, numpy predicate over (x, y)) pairs: calldatasize-like x,
    callvalue-like y, Mythril-shaped lower bounds, alignment and sums."""
    X, Y = CTX.var("mx", XW), CTX.var("my", YW)
    r = random.Random(17)
    out = []
    for _ in range(6):
        a, b, c, k = r.randrange(4, 3000), r.randrange(1, 200), r.randrange(100, 255), r.choice([1, 4, 32])
        cons = [CTX.app("bvugt", X, CTX.const(a, XW)),
                CTX.app("=", CTX.app("bvurem", X, CTX.const(k, XW)), CTX.const(0, XW)),
                CTX.app("bvult", Y, CTX.const(c, YW)),
                CTX.app("bvuge", CTX.app("bvadd", CTX.app("zero_extend", Y, params=(XW - YW,)), X),
                        CTX.const(a + b, XW))]
        pred = (lambda a, b, c, k: lambda x, y: (x > a) & (x % k == 0) & (y < c) & (((x + y) % (1 << XW)) >= a + b))(
            a, b, c, k)
        out.append((cons, pred, X, Y))
    return out


def test_minimize_hint_preserves_the_optimum(mythril, monkeypatch, device):  # noqa: F811
    monkeypatch.setattr(dropin, "_engine", WitnessEngine(dev=device, budget=1 << 20))

    class BV:
        def __init__(self, node):
            self.raw = FakeRaw(node)
            self.node = node

        def size(self):
            return self.node.width

    def uge(a, b):
        return fb(CTX.app("bvuge", CTX.const(a, b.node.width), b.node))
    mythril.mods["mythril.laser.smt"].UGE = uge
    mythril.mods["mythril.laser.smt"].symbol_factory = types.SimpleNamespace(BitVecVal=lambda v, w: v)
    monkeypatch.setattr(z3bridge, "var_name", lambda raw: raw.node.name)
    xs, ys = np.meshgrid(np.arange(1 << XW, dtype=np.int64), np.arange(1 << YW, dtype=np.int64), indexing="ij")
    hinted_n = exact = 0
    for cons, pred, X, Y in _queries():
        ok = pred(xs, ys)
        if not ok.any():
            continue
        opt = int(xs[ok].min())                      # the lexicographic optimum's obj_0
        cs = tuple(fb(c) for c in cons)
        ext = dropin._minimize_hint(cs, (BV(X), BV(Y)), 2000)
        assert ext is not None, "a satisfiable small-domain query gets a device witness"
        bound = ext[-1].raw.node
        assert bound.op == "bvuge" and bound.args[1] is X
        K = bound.args[0].val
        # the witness the bound came from satisfies the constraints, at obj_0 = K
        assert any(bool(ok[K, y]) for y in range(1 << YW))
        assert opt <= K, (opt, K)                    # the optimum survives the hint
        vals = eval_nodes(cons + [bound], {"mx": opt, "my": int(ys[ok][xs[ok] == opt][0])})
        assert all(vals[c.id] for c in cons + [bound])
        cut = 1.0 - (K + 1) / (1 << XW)
        print(f"minimize hint: optimum {opt}, bound {K}, {cut:.1%} of obj_0's domain excluded")
        hinted_n += 1
        exact += K == opt
    assert hinted_n >= 4
    # the descent (model.MINIMIZE_ROUNDS device searches) usually reaches the optimum
    assert exact >= hinted_n // 2, (exact, hinted_n)
