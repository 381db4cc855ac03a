"""The drop-in get_model (mythril_amd/model.py) against a stand-in Mythril.

Neither mythril nor z3 is installable here, so the Mythril
modules get_model touches are replaced by minimal stand-ins with the
reference's semantics (mythril/support/model.py:15-63: timeout clamp,
UnsatError, Python-bool handling, lru_cache of returned models) and the z3
bridge by an IR pass-through whose "z3 re-check" is the oracle.  What is
tested is the drop-in's control flow: GPU answer vs fallback, caching,
error behaviour, rebinding of all three import sites, batched prefetch.
"""
import sys
import types
from functools import lru_cache

import pytest

from mythril_amd import model as dropin
from mythril_amd import z3bridge
from mythril_amd.compiler import Unsupported
from mythril_amd.engine import WitnessEngine
from mythril_amd.ir import Ctx
from mythril_amd.smt2 import Script
from oracle.dag_eval import ArrayVal, eval_nodes
from tests.fakedev import FakeDevice


class UnsatError(Exception):
    pass


class FakeRaw:
    def __init__(self, node):
        self.node = node

    def get_id(self):
        return self.node.id

    def eq(self, other):   # z3.AstRef.eq: structural identity
        return isinstance(other, FakeRaw) and other.node is self.node


class FakeBool:
    def __init__(self, node):
        self.raw = FakeRaw(node)

    def __hash__(self):
        return self.raw.node.id

    def __eq__(self, other):
        return isinstance(other, FakeBool) and other.raw.node.id == self.raw.node.id


class Model:
    def __init__(self, raw):
        self.raw = raw


@pytest.fixture
def mythril(monkeypatch):
    calls = {"reference": 0}
    args = types.SimpleNamespace(solver_timeout=10000, solver_log=None)
    th = types.SimpleNamespace(remaining=100000)
    th.time_remaining = lambda: th.remaining

    @lru_cache(maxsize=2 ** 23)
    def reference_get_model(constraints, minimize=(), maximize=(), enforce_execution_time=True):
        calls["reference"] += 1
        timeout = args.solver_timeout
        if enforce_execution_time:
            timeout = min(timeout, th.time_remaining() - 500)
            if timeout <= 0:
                raise UnsatError
        for c in constraints:
            if type(c) == bool and not c:
                raise UnsatError
        cl = [c for c in constraints if type(c) != bool]
        # stand-in "z3": brute force over the small domains used below
        for v in range(256):
            m = {"x": v, "y": v}
            vals = eval_nodes([c.raw.node for c in cl], m)
            if all(vals[c.raw.node.id] for c in cl):
                return Model(["ref", m])
        raise UnsatError

    mods = {
        "mythril": types.ModuleType("mythril"),
        "mythril.exceptions": types.SimpleNamespace(UnsatError=UnsatError),
        "mythril.support": types.ModuleType("mythril.support"),
        "mythril.support.support_args": types.SimpleNamespace(args=args),
        "mythril.support.model": types.SimpleNamespace(get_model=reference_get_model),
        "mythril.laser": types.ModuleType("mythril.laser"),
        "mythril.laser.ethereum": types.ModuleType("mythril.laser.ethereum"),
        "mythril.laser.ethereum.time_handler": types.SimpleNamespace(time_handler=th),
        "mythril.laser.ethereum.state": types.ModuleType("mythril.laser.ethereum.state"),
        "mythril.laser.ethereum.state.constraints": types.SimpleNamespace(get_model=reference_get_model),
        "mythril.analysis": types.ModuleType("mythril.analysis"),
        "mythril.analysis.solver": types.SimpleNamespace(get_model=reference_get_model),
        "mythril.laser.smt": types.ModuleType("mythril.laser.smt"),
        "mythril.laser.smt.model": types.SimpleNamespace(Model=Model),
    }
    for k, v in mods.items():
        monkeypatch.setitem(sys.modules, k, v)
    mods["mythril"].support = mods["mythril.support"]
    mods["mythril"].analysis = mods["mythril.analysis"]
    mods["mythril"].laser = mods["mythril.laser"]
    mods["mythril.support"].model = mods["mythril.support.model"]
    mods["mythril.analysis"].solver = mods["mythril.analysis.solver"]
    mods["mythril.laser"].ethereum = mods["mythril.laser.ethereum"]
    mods["mythril.laser.ethereum"].state = mods["mythril.laser.ethereum.state"]
    mods["mythril.laser.ethereum.state"].constraints = mods["mythril.laser.ethereum.state.constraints"]

    def to_ir(raws, ctx=None):
        s = Script(ctx or CTX)
        s.asserts = [r.node for r in raws]
        return s

    def confirm(raws, script, w, timeout_ms=2000):
        model = dict(w.values)
        for n, cells in w.arrays.items():
            model[n] = ArrayVal(cells)
        vals = eval_nodes([r.node for r in raws], model)
        return ("z3", model) if all(vals[r.node.id] for r in raws) else None

    monkeypatch.setattr(z3bridge, "to_ir", to_ir)
    monkeypatch.setattr(z3bridge, "model_from_witness", confirm)
    monkeypatch.setattr(dropin, "_engine", WitnessEngine(dev=FakeDevice(chunk=1024), budget=1 << 12))
    monkeypatch.setattr(dropin, "_engine_failed", False)
    monkeypatch.setattr(dropin, "_reference", None)
    dropin._memo.clear()
    dropin.get_model.cache_clear()
    assert dropin.install()
    yield types.SimpleNamespace(calls=calls, args=args, th=th, mods=mods)
    dropin.get_model.cache_clear()


CTX = Ctx()
X = CTX.var("x", 8)


def fb(node):
    return FakeBool(node)


SAT = (fb(CTX.app("bvugt", X, CTX.const(200, 8))), fb(CTX.app("bvult", X, CTX.const(203, 8))))
UNSAT = (fb(CTX.app("bvugt", X, CTX.const(200, 8))), fb(CTX.app("bvult", X, CTX.const(150, 8))))


def test_install_rebinds_all_three_call_sites(mythril):
    m = mythril.mods
    assert m["mythril.support.model"].get_model is dropin.get_model
    assert m["mythril.analysis.solver"].get_model is dropin.get_model
    assert m["mythril.laser.ethereum.state.constraints"].get_model is dropin.get_model


def test_feasible_query_answered_by_gpu_and_confirmed(mythril):
    res = dropin.get_model(SAT)
    assert res.raw[0][0] == "z3" and 200 < res.raw[0][1]["x"] < 203
    assert mythril.calls["reference"] == 0
    assert dropin.STATS["z3_confirmed"] >= 1


def test_unsat_falls_back_to_reference_and_raises(mythril):
    with pytest.raises(UnsatError):
        dropin.get_model(UNSAT)
    assert mythril.calls["reference"] == 1


def test_minimize_always_goes_to_reference(mythril):
    res = dropin.get_model(SAT, minimize=(fb(X),))
    assert res.raw[0] == "ref"


def test_python_false_and_exhausted_budget_raise_unsat(mythril):
    with pytest.raises(UnsatError):
        dropin.get_model(SAT + (False,))
    mythril.th.remaining = 400
    with pytest.raises(UnsatError):
        dropin.get_model((fb(CTX.app("bvugt", X, CTX.const(10, 8))),))


def test_returned_models_are_cached_unsat_is_not(mythril):
    a = dropin.get_model(SAT)
    n = dropin._engine.stats["searches"]
    assert dropin.get_model(SAT) is a
    assert dropin._engine.stats["searches"] == n
    for _ in range(2):
        with pytest.raises(UnsatError):
            dropin.get_model(UNSAT)
    assert mythril.calls["reference"] == 2  # UnsatError is not cached (reference behaviour)


def test_engine_unavailable_or_unsupported_uses_reference(mythril, monkeypatch):
    monkeypatch.setattr(dropin, "_engine", None)
    monkeypatch.setattr(dropin, "_engine_failed", True)
    assert dropin.get_model(SAT).raw[0] == "ref"
    dropin.get_model.cache_clear()
    monkeypatch.setattr(dropin, "_engine_failed", False)
    monkeypatch.setattr(dropin, "_engine", WitnessEngine(dev=FakeDevice(), budget=1 << 10))

    def boom(raws, ctx=None):
        raise Unsupported("z3 op outside the vocabulary")
    monkeypatch.setattr(z3bridge, "to_ir", boom)
    assert dropin.get_model(SAT).raw[0] == "ref"


def test_prefetch_batches_and_feeds_the_memo(mythril):
    sets = [SAT, (fb(CTX.app("=", X, CTX.const(77, 8))),), UNSAT]
    found = dropin.prefetch(sets)
    assert found == 2
    searches = dropin._engine.stats["searches"]
    assert dropin.get_model(sets[1]).raw[0][1]["x"] == 77
    assert dropin._engine.stats["searches"] == searches  # answered from the memo
    assert dropin.STATS["memo_hits"] >= 1


def test_jumpi_successors_searched_in_one_launch(mythril):
    """The plugin's JUMPI post hook defers both successors; the first get_model
    searches them together and the second is answered from the memo."""
    taken = (fb(CTX.app("bvugt", X, CTX.const(100, 8))),)
    fallthrough = (fb(CTX.app("bvule", X, CTX.const(100, 8))),)
    dropin._pending.clear()
    dropin.defer(taken)
    dropin.defer(fallthrough)
    s0 = dropin._engine.stats["searches"]
    assert dropin.get_model(taken).raw[0][1]["x"] > 100
    assert dropin._engine.stats["searches"] == s0 + 1
    assert dropin.get_model(fallthrough).raw[0][1]["x"] <= 100
    assert dropin._engine.stats["searches"] == s0 + 1  # from the memo
    assert not dropin._pending


def test_plugin_registers_rebinding_and_batching_hooks(mythril):
    """WitnessBatchingLaserPlugin.initialize (laser/plugin/interface.py:18) with a
    stand-in LaserEVM: stop_sym_trans prefetch, stop_sym_exec report, JUMPI post
    hook that defers successors."""
    from mythril_amd.mythril_plugin import MI355XWitnessEngine, WitnessBatchingLaserPlugin

    class VM:
        def __init__(self):
            self.laser, self.post, self.open_states = {}, {}, []

        def register_laser_hooks(self, kind, hook):
            self.laser.setdefault(kind, []).append(hook)

        def register_hooks(self, kind, hooks):
            assert kind == "post"
            for op, fs in hooks.items():
                self.post.setdefault(op, []).extend(fs)

    vm = VM()
    plugin = MI355XWitnessEngine()()
    assert isinstance(plugin, WitnessBatchingLaserPlugin)
    plugin.initialize(vm)
    assert set(vm.laser) >= {"stop_sym_trans", "stop_sym_exec"} and "JUMPI" in vm.post
    dropin._pending.clear()
    state = types.SimpleNamespace(world_state=types.SimpleNamespace(constraints=SAT))
    vm.post["JUMPI"][0](state)
    assert dropin._pending == [SAT]
    vm.laser["stop_sym_trans"][0]()  # no open states: a no-op
    dropin._pending.clear()


def test_device_error_falls_back_to_reference(mythril, monkeypatch):
    """an EngineError from the device (failed validation, allocation,
    launch) must never escape get_model; the reference answers instead."""
    from mythril_amd.runtime import EngineError

    class BrokenDevice(FakeDevice):
        def search(self, *a, **k):
            raise EngineError("mg_search failed (-3): out of memory")

    freed = []

    class LeakCheck(FakeDevice):
        n = 0

        def load(self, p):
            LeakCheck.n += 1
            if LeakCheck.n == 2:
                raise EngineError("mg_prog_load failed (-2): pool digit bits > 24")
            dp = super().load(p)
            dp.free = lambda: freed.append(1)
            return dp

    monkeypatch.setattr(dropin, "_engine", WitnessEngine(dev=BrokenDevice(), budget=1 << 10))
    assert dropin.get_model(SAT).raw[0] == "ref"
    assert dropin.STATS["device_errors"] >= 1
    dropin.get_model.cache_clear()
    # a load failure inside a batch frees the programs loaded before it
    monkeypatch.setattr(dropin, "_engine", WitnessEngine(dev=LeakCheck(), budget=1 << 10))
    sets = [SAT, (fb(CTX.app("=", X, CTX.const(77, 8))),)]
    assert dropin.prefetch(sets) == 0
    assert freed == [1]


def test_stale_memo_entry_is_not_used(mythril):
    """z3 reuses the ids of collected ASTs; a memo entry whose ids
    match but whose ASTs differ must not answer."""
    assert dropin.prefetch([SAT]) == 1
    key = dropin.memo_key([c.raw for c in SAT])
    other = (fb(CTX.app("=", X, CTX.const(9, 8))), fb(CTX.app("bvult", X, CTX.const(10, 8))))
    raws_other = [c.raw for c in other]
    # pretend z3 handed the same ids to different ASTs
    dropin._memo[dropin.memo_key(raws_other)] = dropin._memo[key]
    assert dropin._memo_get(raws_other, dropin.memo_key(raws_other)) is None
    assert dropin.memo_key(raws_other) not in dropin._memo
    res = dropin.get_model(other)
    assert res.raw[0][1]["x"] == 9


def test_repeated_miss_skips_the_device(mythril, monkeypatch):
    """UNSAT is never cached by get_model (reference behaviour), so LASER asks an
    infeasible set again: the second time the device is skipped and z3 answers
    directly (same results).  A one-conjunct extension is searched again by
    default (its re-harvested pools may pin a value the parent lacked: ADVICE
    r2), and skipped only with MYTHRIL_AMD_SKIP_MISS_PREFIX=1."""
    dropin._misses.clear()
    s0 = dropin._engine.stats["searches"]
    with pytest.raises(UnsatError):
        dropin.get_model(UNSAT)
    assert dropin._engine.stats["searches"] == s0 + 1
    with pytest.raises(UnsatError):
        dropin.get_model(UNSAT)
    assert dropin._engine.stats["searches"] == s0 + 1
    ext = UNSAT + (fb(CTX.app("bvugt", X, CTX.const(3, 8))),)
    with pytest.raises(UnsatError):
        dropin.get_model(ext)
    assert dropin._engine.stats["searches"] == s0 + 2      # default: the extension is searched
    monkeypatch.setattr(dropin, "SKIP_EXTENSIONS_OF_MISSES", True)
    ext2 = UNSAT + (fb(CTX.app("bvugt", X, CTX.const(4, 8))),)
    with pytest.raises(UnsatError):
        dropin.get_model(ext2)
    assert dropin._engine.stats["searches"] == s0 + 2      # opt-in: skipped
    assert dropin.STATS["miss_skips"] >= 2
    assert mythril.calls["reference"] == 4
    # a satisfiable set is still searched
    assert dropin.get_model(SAT).raw[0][0] == "z3"


def test_extension_that_pins_a_value_hits_where_its_parent_missed(mythril):
    """x > 250 misses in a tiny budget of generated candidates, but
    the extension x == 251 gets an exact pool and the device answers it."""
    dropin._misses.clear()
    parent = (fb(CTX.app("bvugt", X, CTX.const(250, 8))), fb(CTX.app("bvult", X, CTX.const(252, 8))))
    ext = parent + (fb(CTX.app("=", X, CTX.const(251, 8))),)
    praws = [c.raw for c in parent]
    dropin._record_miss(praws, dropin.memo_key(praws))     # as if the device had missed the parent
    r = dropin.get_model(ext)
    assert r.raw[0][0] == "z3" and r.raw[0][1]["x"] == 251


def test_minimize_hint_bounds_only_the_first_objective(mythril, monkeypatch):
    """Opt-in minimize assistance (analysis/solver.py:216-256): a device witness
    adds obj_0 <= witness(obj_0) to the set z3's Optimize gets; the objectives
    themselves are untouched.  Off by default (the report's transaction data
    could differ), and a minimize query without it goes to z3 unchanged."""
    seen = []
    ref = dropin._reference

    def recording(constraints, minimize=(), maximize=(), enforce_execution_time=True):
        seen.append((constraints, minimize))
        return Model(["ref"])
    monkeypatch.setattr(dropin, "_reference", recording)
    Y = CTX.var("y", 8)

    class BV:
        def __init__(self, node):
            self.raw = FakeRaw(node)
            self.node = node

        def size(self):
            return self.node.width

    def uge(a, b):
        return fb(CTX.app("bvuge", CTX.const(a, 8), b.node))
    mythril.mods["mythril.laser.smt"].UGE = uge
    mythril.mods["mythril.laser.smt"].symbol_factory = types.SimpleNamespace(BitVecVal=lambda v, w: v)
    monkeypatch.setattr(z3bridge, "var_name", lambda raw: raw.node.name)
    objs = (BV(X), BV(Y))
    dropin.get_model(SAT, minimize=objs)
    assert seen[-1][0] == SAT                        # default: unchanged
    monkeypatch.setattr(dropin, "MINIMIZE_HINTS", True)
    dropin.get_model.cache_clear()
    dropin.get_model(SAT, minimize=objs)
    hinted, mins = seen[-1]
    assert mins == objs and len(hinted) == len(SAT) + 1
    bound = hinted[-1].raw.node
    assert bound.op == "bvuge" and bound.args[1] is X and 200 < bound.args[0].val < 203
    assert dropin.STATS["minimize_hints"] >= 1
    monkeypatch.setattr(dropin, "_reference", ref)


def test_prefetch_miss_on_a_shortened_budget_is_searched_again(mythril, monkeypatch):
    """a batch divides the op budget over its programs, so a miss in
    it is recorded (and later skipped by get_model) only when the batch gave the
    set at least the candidates get_model's own launch would."""
    from mythril_amd import engine as engine_mod
    monkeypatch.setattr(engine_mod, "MIN_CANDIDATES", 16)
    eng = dropin._engine
    unsat2 = (fb(CTX.app("bvugt", X, CTX.const(240, 8))), fb(CTX.app("bvult", X, CTX.const(10, 8))))
    q = engine_mod.prepare([c.raw.node for c in UNSAT], CTX)
    monkeypatch.setattr(eng, "op_budget", q.ops_per_eval * eng.budget)   # one set alone: the full budget
    dropin._misses.clear()
    assert dropin.prefetch([UNSAT, unsat2]) == 0
    assert not dropin._misses                           # each got about half: nothing recorded
    s0 = eng.stats["searches"]
    with pytest.raises(UnsatError):
        dropin.get_model(UNSAT)
    assert eng.stats["searches"] == s0 + 1              # searched again, on its own budget
    monkeypatch.setattr(eng, "op_budget", None)         # every launch gets the full budget
    dropin._misses.clear()
    assert dropin.prefetch([UNSAT, unsat2]) == 0
    assert len(dropin._misses) == 2


def test_minimize_hint_needs_a_confirmed_witness(mythril, monkeypatch):
    """the hint becomes a hard bound, so a witness the reference
    solver does not confirm gives no hint at all."""
    Y = CTX.var("y", 8)

    class BV:
        def __init__(self, node):
            self.raw = FakeRaw(node)
            self.node = node

        def size(self):
            return self.node.width
    monkeypatch.setattr(z3bridge, "var_name", lambda raw: raw.node.name)
    monkeypatch.setattr(z3bridge, "model_from_witness", lambda *a, **k: None)
    assert dropin._minimize_hint(SAT, (BV(X), BV(Y)), 2000) is None


def test_witness_layout_mismatch_falls_back_to_reference(mythril, monkeypatch):
    """materialize's layout check raises EngineError, which get_model
    turns into a z3 answer instead of an exception in LASER."""
    from mythril_amd import engine as engine_mod
    from mythril_amd.compiler import compile_program
    real = engine_mod.prepare
    monkeypatch.setattr(FakeDevice, "witness_leaves", None)   # the traced path (witness program)

    def broken(conj, ctx, **kw):
        q = real(conj, ctx, **kw)
        q._trace = compile_program([], leaf_specs={})     # no leaves: layout differs
        return q
    monkeypatch.setattr(engine_mod, "prepare", broken)
    assert dropin.get_model(SAT).raw[0] == "ref"
    assert dropin.STATS["device_errors"] >= 1


def test_constant_cells_materialise_from_leaves(mythril, monkeypatch):
    """A witness is read in the search's own synchronisation (mg_search_end
    evaluates the witness program at the found index; round 6): no witness
    call of its own.  With MYTHRIL_AMD_WITNESS_IN_LAUNCH=0, a witness whose
    array cells all have constant indices is read from the search program's
    leaves (mg_witness_leaves), without a witness program."""
    from mythril_amd import engine as engine_mod
    dev = dropin._engine.dev
    n0, b0 = getattr(dev, "witness_leaf_calls", 0), getattr(dev, "begin_calls", 0)
    res = dropin.get_model(SAT)
    assert res.raw[0][0] == "z3"
    assert getattr(dev, "witness_leaf_calls", 0) == n0 and getattr(dev, "begin_calls", 0) == b0 + 1
    monkeypatch.setattr(engine_mod, "WITNESS_IN_LAUNCH", False)
    dropin.get_model.cache_clear()
    dropin._memo.clear()
    res = dropin.get_model(SAT)
    assert res.raw[0][0] == "z3"
    assert getattr(dev, "witness_leaf_calls", 0) == n0 + 1


def test_slow_recheck_is_counted_and_logged(mythril, monkeypatch, caplog):
    """VERDICT r4 item 8 (SURVEY §7 hard part 5): the z3 re-check runs under
    the pinned budget first; a witness z3 confirms only with more time (it
    answered unknown under the pinned budget) is still returned, and counted
    and logged, because the reference's check of the unpinned formula may
    have timed out there."""
    calls = []

    def slow_confirm(raws, script, w, timeout_ms=2000):
        calls.append(timeout_ms)
        if timeout_ms <= dropin.PINNED_CHECK_MS:
            z3bridge._last.info = {"result": "unknown", "ms": timeout_ms}
            return None
        z3bridge._last.info = {"result": "sat", "ms": 1.0}
        return ("z3", dict(w.values))
    monkeypatch.setattr(z3bridge, "model_from_witness", slow_confirm)
    n0 = dropin.STATS.get("slow_rechecks", 0)
    with caplog.at_level("WARNING"):
        res = dropin.get_model(SAT)
    assert res.raw[0][0] == "z3"
    # the second check gets the rest of the query's budget
    assert calls == [dropin.PINNED_CHECK_MS, mythril.args.solver_timeout - dropin.PINNED_CHECK_MS]
    assert dropin.STATS["slow_rechecks"] == n0 + 1
    assert "pinned re-check budget" in caplog.text
    # MYTHRIL_AMD_SLOW_RECHECK=reference: the reference solver answers instead
    dropin.get_model.cache_clear()
    dropin._memo.clear()
    calls.clear()
    monkeypatch.setattr(z3bridge, "SLOW_RECHECK", "reference")
    assert dropin.get_model(SAT).raw[0] == "ref"
    assert calls == [dropin.PINNED_CHECK_MS]
    monkeypatch.setattr(z3bridge, "SLOW_RECHECK", "confirm")
    # an unsat answer under the pinned budget is final: no second check
    dropin.get_model.cache_clear()
    dropin._memo.clear()
    calls.clear()

    def refuted(raws, script, w, timeout_ms=2000):
        calls.append(timeout_ms)
        z3bridge._last.info = {"result": "unsat", "ms": 1.0}
        return None
    monkeypatch.setattr(z3bridge, "model_from_witness", refuted)
    assert dropin.get_model(SAT).raw[0] == "ref"
    assert calls == [dropin.PINNED_CHECK_MS]
