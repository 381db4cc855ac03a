"""Drop-in replacement for ``mythril.support.model.get_model``.

Same signature, same ``@lru_cache(maxsize=2**23)``, same error behaviour as
``mythril/support/model.py:15-63``:

* the solver timeout is clamped to the remaining execution budget and
  ``UnsatError`` is raised when it is <= 0 (``:26-31``);
* a Python ``False`` constraint raises ``UnsatError`` (``:32-34``);
* a ``Constraints`` object is expanded with the keccak conditions via
  ``get_all_constraints()`` (``:35-36``); Python bools are dropped (``:37``);
* ``--solver-log`` dumps are written exactly as the reference writes them
  (``:45-56``), whether or not the GPU answers;
* only *returned models* are cached; ``UnsatError`` is never cached.

New: when ``minimize == maximize == ()`` (feasibility-only queries: LASER's
``is_possible`` pruning, the detection modules' checks)
and the formula lowers to the witness engine, a batched GPU search runs first.
A witness is re-checked by z3 on the exact same constraints and z3's model of
that check is returned.  On a miss, an unsupported formula, an unavailable
engine, or a witness z3 does not confirm, the *unchanged* reference function
answers (``minimize`` queries from ``get_transaction_sequence``,
``analysis/solver.py:68``, always go to the reference).
"""
from __future__ import annotations

import logging
import os
import threading
from functools import lru_cache
from pathlib import Path
from typing import Callable, Dict, Optional

from .compiler import Unsupported

log = logging.getLogger(__name__)

STATS: Dict[str, int] = {"queries": 0, "gpu_attempts": 0, "gpu_witnesses": 0, "z3_confirmed": 0,
                         "unsupported": 0, "fallbacks": 0, "memo_hits": 0}

# injection points (set by install(); replaced by tests)
_reference: Optional[Callable] = None   # the reference get_model, uncached (__wrapped__)
_engine = None
_engine_lock = threading.Lock()
_engine_failed = False
_memo: Dict[tuple, tuple] = {}          # z3 AST-id key -> (raws, witness, script)
MEMO_MAX = 1 << 16
_pending: list = []                     # successor constraint sets deferred by the JUMPI hook
PENDING_MAX = 64
# Misses: get_model never caches UNSAT (the reference raises UnsatError, which
# lru_cache does not keep), so LASER asks the same infeasible set again and
# again.  A set the device already searched without a witness skips the device
# the next time (z3 answers, as it would anyway).  Extensions of a missed set
# by one conjunct are searched again by default: prepare() re-harvests the
# pools from the extended set, so a successor that pins a value (x == K) gets
# an exact domain and can hit where its parent missed.
# MYTHRIL_AMD_SKIP_MISS_PREFIX=1 skips them too (less device time, fewer hits).
_misses: Dict[tuple, list] = {}          # z3 AST-id key -> raws (kept alive, eq-confirmed)
MISS_MAX = 1 << 14
SKIP_EXTENSIONS_OF_MISSES = os.environ.get("MYTHRIL_AMD_SKIP_MISS_PREFIX", "0") == "1"


def _env():
    from mythril.exceptions import UnsatError
    from mythril.laser.ethereum.time_handler import time_handler
    from mythril.support.support_args import args
    return args, time_handler, UnsatError


def engine():
    """The process's WitnessEngine, or None if the HIP engine is unavailable."""
    global _engine, _engine_failed
    if _engine is None and not _engine_failed:
        with _engine_lock:
            if _engine is None and not _engine_failed:
                if os.environ.get("MYTHRIL_AMD_DISABLE"):
                    _engine_failed = True
                    return None
                try:
                    from .engine import WitnessEngine
                    dev = int(os.environ.get("LOCAL_RANK", os.environ.get("MYTHRIL_AMD_DEVICE", "0")))
                    budget = int(os.environ.get("MYTHRIL_AMD_BUDGET", str(1 << 22)))
                    from .engine import DEFAULT_ASMJIT_MIN_OPS, DEFAULT_OP_BUDGET
                    op_budget = int(os.environ.get("MYTHRIL_AMD_OP_BUDGET", str(DEFAULT_OP_BUDGET)))
                    asm_min = int(os.environ.get("MYTHRIL_AMD_ASMJIT_MIN_OPS", str(DEFAULT_ASMJIT_MIN_OPS)))
                    ndev = int(os.environ.get("MYTHRIL_AMD_DEVICES", "1"))
                    multi = None
                    if ndev > 1:   # one process over several GPUs (multidev.py)
                        from .multidev import MultiDevice
                        multi = MultiDevice.open(range(ndev))
                    _engine = WitnessEngine(device=dev, budget=budget, op_budget=op_budget, dev=multi,
                                            asmjit_min_ops=asm_min)
                except Exception as e:  # EngineUnavailable / EngineError
                    log.warning("MI355X witness engine unavailable (%s); using z3 only", e)
                    _engine_failed = True
    return _engine


def memo_key(raws) -> tuple:
    return tuple(r.get_id() for r in raws)


def _known_miss(raws, key) -> bool:
    for k, rs in ((key, raws), (key[:-1], raws[:-1]) if SKIP_EXTENSIONS_OF_MISSES and len(raws) > 1 else (None, None)):
        if k is None:
            continue
        kept = _misses.get(k)
        if kept is not None and len(kept) == len(rs) and all(a is b or a.eq(b) for a, b in zip(kept, rs)):
            return True
    return False


def _record_miss(raws, key) -> None:
    if len(_misses) >= MISS_MAX:
        _misses.clear()
    _misses[key] = list(raws)


def _memo_get(raws, key):
    """The memo entry for these ASTs.  z3 reuses the ids of collected ASTs, so
    an id match is confirmed structurally (``eq``) against the ASTs the entry
    keeps alive; a stale entry is dropped."""
    hit = _memo.get(key)
    if hit is None:
        return None
    kept = hit[0]
    if len(kept) == len(raws) and all(a is b or a.eq(b) for a, b in zip(kept, raws)):
        return hit
    del _memo[key]
    return None


def _solver_log(constraints, minimize, maximize, args, timeout):
    """Write the .smt2 dump exactly as mythril/support/model.py:45-56 does."""
    from mythril.laser.smt import Optimize
    s = Optimize()
    s.set_timeout(timeout)
    for c in constraints:
        s.add(c)
    for e in minimize:
        s.minimize(e)
    for e in maximize:
        s.maximize(e)
    Path(args.solver_log).mkdir(parents=True, exist_ok=True)
    key = tuple(list(constraints) + list(minimize) + list(maximize)
                + [len(constraints), len(minimize), len(maximize)])
    with open(args.solver_log + f"/{abs(hash(key))}.smt2", "w") as f:
        f.write(s.sexpr())


def _gpu_model(constraints, timeout):
    from . import z3bridge
    from .runtime import EngineError
    raws = [c.raw for c in constraints]
    key = memo_key(raws)
    hit = _memo_get(raws, key)
    if hit is None and _pending:
        # the JUMPI successors LASER is about to prune one by one (svm.py:287-292):
        # search all of them in one launch, then answer this one from the memo
        batch = _pending[:]
        _pending.clear()
        STATS["batched_prefetches"] = STATS.get("batched_prefetches", 0) + 1
        prefetch(batch)
        hit = _memo_get(raws, key)
    if hit is not None:
        STATS["memo_hits"] += 1
        _, witness, script = hit
    else:
        eng = engine()
        if eng is None:
            return None
        if _known_miss(raws, key):
            STATS["miss_skips"] = STATS.get("miss_skips", 0) + 1
            return None
        try:
            script = z3bridge.to_ir(raws)
            from .engine import prepare
            q = prepare(script.asserts, script.ctx)
        except (Unsupported, RecursionError, ValueError, KeyError) as e:
            STATS["unsupported"] += 1
            log.debug("witness engine: unsupported formula (%s)", e)
            return None
        except Exception as e:   # z3 printing/parsing trouble: fail closed to the reference
            STATS["unsupported"] += 1
            log.warning("witness engine: could not translate the query (%s)", e)
            return None
        STATS["gpu_attempts"] += 1
        try:
            witness = eng.search([q])[0]
        except EngineError as e:
            # a device-side failure (validation, allocation, launch) never escapes:
            # the reference answers, exactly as without the engine
            STATS["device_errors"] = STATS.get("device_errors", 0) + 1
            log.warning("witness engine: device error (%s); z3 answers", e)
            return None
        if witness is None:
            _record_miss(raws, key)
    if witness is None:
        return None
    STATS["gpu_witnesses"] += 1
    try:
        zm, slow = z3bridge.recheck(raws, script, witness, timeout, PINNED_CHECK_MS)
    except Exception as e:   # fail closed: the reference answers
        STATS["recheck_errors"] = STATS.get("recheck_errors", 0) + 1
        log.warning("witness engine: z3 re-check failed (%s); z3 answers", e)
        return None
    if zm is None:
        return None
    if slow:
        # visible divergence risk (SURVEY §7 hard part 5): z3 needed more than
        # the pinned budget even with every symbol pinned, so the reference's
        # check of the unpinned formula may well have timed out (unknown ->
        # UnsatError, a pruned state) where this path answers sat
        STATS["slow_rechecks"] = STATS.get("slow_rechecks", 0) + 1
        log.warning("witness engine: z3 confirmed a GPU witness only after the pinned re-check budget "
                    "(%d ms); the reference solver may have answered unknown on this query", PINNED_CHECK_MS)
    STATS["z3_confirmed"] += 1
    from mythril.laser.smt.model import Model
    return Model([zm])


# z3's budget for the re-check of a witness with every symbol pinned; a
# re-check that needs more is retried with the query's timeout and counted
# (STATS["slow_rechecks"], logged)
PINNED_CHECK_MS = int(os.environ.get("MYTHRIL_AMD_PINNED_CHECK_MS", "250"))
MINIMIZE_HINTS = os.environ.get("MYTHRIL_AMD_MINIMIZE_HINTS", "0") == "1"
MINIMIZE_ROUNDS = int(os.environ.get("MYTHRIL_AMD_MINIMIZE_ROUNDS", "8"))   # device descent searches


def _walk(roots):
    from .ir import topo
    return topo(list(roots))


def _minimize_hint(constraints, minimize, timeout):
    """Minimize assistance (``analysis/solver.py:216-256``),
    OFF by default (``MYTHRIL_AMD_MINIMIZE_HINTS=1``).

    ``get_transaction_sequence`` asks z3's Optimize for lexicographically
    minimal ``calldatasize``/``call_value`` per transaction.  A device witness
    of the same constraints bounds the FIRST objective from above: adding
    ``obj_0 <= witness(obj_0)`` cannot change the optimum (the optimal model
    satisfies it), only prune z3's search.  The bound is tightened by up to
    MINIMIZE_ROUNDS more searches with ``obj_0 <=u target`` added, the target
    halving the gap to the lowest value not yet ruled out by a miss (a miss
    proves nothing, it only moves the target up).  Later objectives get no bound (the
    witness need not be optimal in obj_0, so its later values bound nothing in
    the lexicographic order).  The optimum is preserved, but z3 may return a
    different model with the same objective values, i.e. different transaction
    data in the issue report: hence opt-in.  Returns the extended constraint
    collection, or None (no witness, objective not a plain variable, engine
    unavailable)."""
    if not minimize:
        return None
    cl = constraints if type(constraints) == tuple else constraints.get_all_constraints()
    cl = [c for c in cl if type(c) != bool]
    raws = [c.raw for c in cl]
    eng = engine()
    if eng is None:
        return None
    from . import z3bridge
    from .runtime import EngineError
    obj = minimize[0]
    name = z3bridge.var_name(obj.raw)
    if name is None:
        return None
    def confirmed(w) -> bool:
        # the bound becomes a hard constraint of z3's Optimize: a value the
        # reference solver does not confirm on the unextended set is never used
        # (the verdict and the values come from different programs)
        try:
            return z3bridge.model_from_witness(raws, script, w, timeout) is not None
        except Exception as e:   # noqa: BLE001 - fail closed: no hint
            log.warning("witness engine: z3 re-check of a minimize hint failed (%s)", e)
            return False

    try:
        script = z3bridge.to_ir(raws)
        from .engine import prepare
        q = prepare(script.asserts, script.ctx)
        w = eng.search([q])[0]
        if w is None or name not in w.values or not confirmed(w):
            return None
        best = w.values[name]
        # descent: search again below the best value so far, aiming at half of
        # it first (each round adds obj_0 <u target; a miss proves nothing, so
        # the target moves back up towards the best witness)
        var = next((n for n in _walk(script.asserts) if n.op == "var" and n.name == name), None)
        lo = 0
        for _ in range(MINIMIZE_ROUNDS if var is not None else 0):
            if best <= lo:
                break
            target = lo + (best - lo) // 2
            extra = script.ctx.app("bvule", var, script.ctx.const(target, var.width))
            w2 = eng.search([prepare(list(script.asserts) + [extra], script.ctx)])[0]
            if w2 is not None and name in w2.values and w2.values[name] <= target and confirmed(w2):
                best = w2.values[name]
            else:
                lo = target + 1
        STATS["minimize_rounds"] = STATS.get("minimize_rounds", 0) + 1
    except (Unsupported, RecursionError, ValueError, KeyError, EngineError):
        return None
    from mythril.laser.smt import UGE, symbol_factory
    bound = UGE(symbol_factory.BitVecVal(best, obj.size()), obj)
    STATS["minimize_hints"] = STATS.get("minimize_hints", 0) + 1
    if type(constraints) == tuple:
        return constraints + (bound,)
    import copy
    ext = copy.copy(constraints)
    ext.append(bound)
    return ext


@lru_cache(maxsize=2 ** 23)
def get_model(constraints, minimize=(), maximize=(), enforce_execution_time=True):
    """mythril.support.model.get_model with a GPU witness fast path (see module doc)."""
    args, time_handler, UnsatError = _env()
    STATS["queries"] += 1
    timeout = args.solver_timeout
    if enforce_execution_time:
        timeout = min(timeout, time_handler.time_remaining() - 500)
        if timeout <= 0:
            raise UnsatError
    for constraint in constraints:
        if type(constraint) == bool and not constraint:
            raise UnsatError
    if minimize == () and maximize == ():
        cl = constraints if type(constraints) == tuple else constraints.get_all_constraints()
        cl = [c for c in cl if type(c) != bool]
        model = _gpu_model(cl, timeout)
        if model is not None:
            if args.solver_log:
                _solver_log(cl, minimize, maximize, args, timeout)
            return model
    STATS["fallbacks"] += 1
    if MINIMIZE_HINTS and minimize and not maximize:
        hinted = _minimize_hint(constraints, minimize, timeout)
        if hinted is not None:
            return _reference(hinted, minimize, maximize, enforce_execution_time)
    return _reference(constraints, minimize, maximize, enforce_execution_time)


def defer(constraints) -> None:
    """Queue a fresh state's constraint set (the plugin's JUMPI post hook, run
    on each successor before LASER's per-step prune): the next memo miss in
    get_model searches every queued set in the same launch."""
    if len(_pending) < PENDING_MAX:
        _pending.append(constraints)


def prefetch(constraint_sets) -> int:
    """Batch feasibility search for many constraint sets in one launch (LaserEVM
    open states at a transaction boundary, svm.py:216-223); fills the memo that
    get_model consults.  Returns the number of witnesses found."""
    eng = engine()
    if eng is None:
        return 0
    from . import z3bridge
    from .engine import prepare
    from .runtime import EngineError
    items = []
    for cs in constraint_sets:
        try:
            cl = cs if type(cs) == tuple else cs.get_all_constraints()
            raws = [c.raw for c in cl if type(c) != bool]
            key = memo_key(raws)
            if _memo_get(raws, key) is not None:
                continue
            script = z3bridge.to_ir(raws)
            items.append((key, raws, script, prepare(script.asserts, script.ctx)))
        except (Unsupported, RecursionError, ValueError, KeyError):
            STATS["unsupported"] += 1
        except Exception as e:   # noqa: BLE001 - z3 printing/parsing trouble: that set goes to z3
            STATS["unsupported"] += 1
            log.warning("witness engine: could not translate a batched query (%s)", e)
    if not items:
        return 0
    qs = [q for *_, q in items]
    try:
        found = eng.search(qs)
    except EngineError as e:
        STATS["device_errors"] = STATS.get("device_errors", 0) + 1
        log.warning("witness engine: device error in batched prefetch (%s)", e)
        return 0
    # a batch splits the op budget over its programs, so each got at most the
    # candidates get_model's own launch would give it
    count_of = getattr(eng, "launch_count", None)
    batch_count = count_of(qs) if count_of else None
    n = 0
    for (key, raws, script, q), w in zip(items, found):
        if w is not None:
            if len(_memo) >= MEMO_MAX:
                _memo.clear()
            _memo[key] = (raws, w, script)
            n += 1
        elif batch_count is not None and batch_count >= count_of([q]):
            # searched with the budget get_model would use: its is_possible
            # goes straight to the reference instead of searching again.  A
            # miss on a shortened budget is not recorded: get_model searches
            # that set again with its full budget.
            _record_miss(raws, key)
    return n


def install() -> bool:
    """Rebind every import site of get_model (SURVEY.md §8b "Who calls it")."""
    global _reference
    try:
        import mythril.analysis.solver as a_solver
        import mythril.laser.ethereum.state.constraints as l_constraints
        import mythril.support.model as s_model
    except ImportError:
        return False
    if getattr(s_model.get_model, "__module__", "") == __name__:
        return True
    ref = s_model.get_model
    _reference = getattr(ref, "__wrapped__", ref)
    s_model.get_model = get_model
    a_solver.get_model = get_model
    l_constraints.get_model = get_model
    log.info("MI355X witness engine installed behind mythril get_model")
    return True
