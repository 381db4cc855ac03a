"""The z3 AST walker (mythril_amd/z3walk.py) and the per-conjunct cache
(z3bridge.ConjunctCache) against the text route, with the stand-in z3 of
tests/fakez3.py (z3 is absent here and on the box: parity with the real z3
API stays unpinned).

* the walker builds exactly the terms the SMT-LIB parser builds from the
  same conjuncts' text: the same IR nodes in one context, on every query of
  both corpora;
* in LASER's query order (tests/laser_concolic.py runs), the cached route
  (walker + per-conjunct lowering / congruence / harvest memos in the
  long-lived context) gives byte-identical programs to the whole-set text
  route, and translates each conjunct once;
* an operator the walker does not know falls back to printing."""
import gzip
import os
import sys

import numpy as np
import pytest

from mythril_amd import z3bridge, z3walk
from mythril_amd.compiler import Unsupported
from mythril_amd.engine import prepare
from mythril_amd.ir import Ctx
from mythril_amd.smt2 import parse_file, parse_script, to_smt2
from tests import fakez3

HERE = os.path.dirname(os.path.abspath(__file__))


def _corpus_files():
    out = []
    for d in ("solver_log", "laser"):
        base = os.path.join(HERE, "golden", d)
        out += [os.path.join(base, f) for f in sorted(os.listdir(base)) if ".smt2" in f]
    return out


def test_walker_builds_the_parsers_terms():
    files = _corpus_files()
    assert len(files) > 800
    for f in files[::3]:
        s = parse_file(f)
        z = fakez3.module()
        ctx = Ctx()
        w = z3walk.Z3Walker(z, ctx)
        walked = [w.term(z.ast(n)) for n in s.asserts]
        parsed = parse_script(to_smt2(s.asserts), ctx).asserts
        assert all(a is b for a, b in zip(walked, parsed)), f
        assert set(w.decls) <= set(parse_script(to_smt2(s.asserts)).decls)


def test_walker_memoises_by_ast():
    c = Ctx()
    x = c.var("x", 256)
    word = c.app("concat", *[c.app("extract", x, params=(8 * i + 7, 8 * i)) for i in range(31, -1, -1)])
    a1 = c.app("bvult", word, c.const(5, 256))
    a2 = c.app("bvugt", word, c.const(1, 256))
    z = fakez3.module()
    w = z3walk.Z3Walker(z, Ctx())
    w.term(z.ast(a1))
    n = len(w.memo)
    w.term(z.ast(a2))
    assert len(w.memo) == n + 2        # the new comparison and its constant: the word is shared


def test_unknown_operator_falls_back_to_printing(monkeypatch):
    z = fakez3.module()
    monkeypatch.setitem(sys.modules, "z3", z)
    c = Ctx()
    x = c.var("x", 8)
    t = c.app("bvugt", c.app("bvnand", x, c.const(3, 8)), c.const(1, 8))
    delattr(z, "Z3_OP_BNAND")          # a z3 build without that kind name
    cache = z3bridge.ConjunctCache()
    s = cache.to_ir([z.ast(t)])
    assert cache.stats["prints"] == 1 and cache.stats["walked"] == 0
    assert s.asserts[0].op == "bvugt" and s.asserts[0].args[0].op == "bvnand"


def _program_bytes(p):
    return b"|".join(np.asarray(x, dtype=np.uint32).tobytes() for x in (p.code, p.consts, p.leaves)) + \
        repr(p.ops_per_eval).encode()


@pytest.mark.parametrize("contract", ["underflow", "calls", "environments", "symbolic_exec_bytecode"])
def test_cached_route_gives_the_same_programs_in_laser_order(monkeypatch, contract):
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))
    from make_laser_corpus import SCENARIOS, load_code, scenario_balances
    from tests.laser_concolic import run_sequence
    z = fakez3.module()
    monkeypatch.setitem(sys.modules, "z3", z)
    name, txs, *opt = SCENARIOS[contract][0]
    opts = opt[0] if opt else {}
    _, run = run_sequence(load_code(contract), txs, storage=opts.get("storage"), balances=scenario_balances(opts))
    cache = z3bridge.ConjunctCache()
    seen = set()
    for q in run.queries:
        whole = parse_script(to_smt2(q.constraints))
        pw = prepare(whole.asserts, whole.ctx).program
        sc = cache.to_ir([z.ast(n) for n in q.constraints])
        pc = prepare(sc.asserts, sc.ctx).program
        assert _program_bytes(pw) == _program_bytes(pc), (contract, q.pc, q.kind)
        seen.update(n.id for n in q.constraints)
    assert cache.stats["walked"] == len(seen) and cache.stats["prints"] == 0
    assert z.calls["sexpr"] == 0


def test_decls_of_a_long_lived_cache_pin_the_witness(monkeypatch):
    """model_from_witness looks the witness's names up in the cache's
    declaration table (every symbol of the process): scalars, cells and
    function points of this query only."""
    from mythril_amd.engine import Witness
    from tests.test_z3bridge import FakeZ3
    fz = FakeZ3()
    monkeypatch.setitem(sys.modules, "z3", fz)
    script = parse_script(gzip.open(_corpus_files()[-1], "rt").read())
    script.decls = dict(script.decls)
    from mythril_amd.smt2 import Decl, Sort
    script.decls["unrelated"] = Decl("unrelated", [], Sort("bv", 256))
    name = next(n for n, d in script.decls.items() if not d.args and d.sort.kind == "bv" and n != "unrelated")
    assert z3bridge.model_from_witness(["raw"], script, Witness(0, {name: 5, "cd@3": 1})) is not None
    pinned = [p for p in fz.pins if isinstance(p, tuple) and p[0] == "pin"]
    assert [p[1] for p in pinned] == [name]


def test_sort_conflicts_reset_once_and_fail_closed(monkeypatch):
    """one name with two sorts across queries resets the cache once
    and translates the new set; a set that uses one name with two sorts
    itself is refused after that one retry (the reference solver answers),
    not retried until a RecursionError."""
    z = fakez3.module()
    monkeypatch.setitem(sys.modules, "z3", z)
    c1, c2 = Ctx(), Ctx()
    a8 = c1.app("bvugt", c1.var("x", 8), c1.const(1, 8))
    a16 = c2.app("bvugt", c2.var("x", 16), c2.const(1, 16))
    cache = z3bridge.ConjunctCache()
    s = cache.to_ir([z.ast(a8)])
    assert s.asserts[0].args[0].width == 8
    s = cache.to_ir([z.ast(a16)])
    assert s.asserts[0].args[0].width == 16 and cache.stats["resets"] <= 1
    resets = cache.stats["resets"]
    with pytest.raises(Exception) as ei:
        cache.to_ir([z.ast(a8), z.ast(a16)])
    assert not isinstance(ei.value, RecursionError)
    assert cache.stats["resets"] <= resets + 1
