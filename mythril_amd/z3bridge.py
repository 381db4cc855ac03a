"""z3 <-> witness-engine glue (used only inside a Mythril process, where z3 exists).

* ``to_ir``: a list of z3 ``BoolRef`` -> the solver script text (exactly the
  ``Optimize.sexpr()`` form ``--solver-log`` writes, ``mythril/support/model.py:45-56``)
  -> :mod:`mythril_amd.smt2` -> IR conjuncts.
* ``model_from_witness``: re-checks a GPU witness *in z3* on the exact same
  constraints (including the current keccak conditions) by pinning every free
  symbol / array cell / function application to the witness values, and
  returns z3's model of that query — so the caller gets a genuine
  ``z3.ModelRef`` (what ``Optimize.model()`` returns, ``solver.py:68-77``),
  or ``None`` if z3 does not confirm it (then the reference path runs).
"""
from __future__ import annotations

import logging
import os
import threading
import time
from typing import List, Optional, Sequence, Tuple

from .compiler import Unsupported
from .engine import Witness
from .ir import BOOL, Ctx
from .smt2 import Script, parse_script

log = logging.getLogger(__name__)


def _z3():
    import z3  # noqa: WPS433 - only available inside Mythril's environment
    return z3


def var_name(raw) -> Optional[str]:
    """The declaration name of a z3 constant (an uninterpreted 0-ary symbol), else None."""
    try:
        if raw.num_args() == 0 and raw.decl().kind() == _z3().Z3_OP_UNINTERPRETED:
            return raw.decl().name()
    except Exception:
        return None
    return None


def solver_sexpr(raws: Sequence) -> str:
    """z3's SMT-LIB text of a set of assertions (``Solver.sexpr()``: the
    declarations of the symbols they use, one ``assert`` each, shared
    subterms let-bound; the text ``--solver-log`` writes)."""
    z3 = _z3()
    s = z3.Solver()
    s.add(list(raws))
    return s.sexpr()


class ConjunctCache:
    """Per-conjunct translation cache keyed by z3 AST id.

    A LASER successor's constraint set is its parent's plus one conjunct
    (``instructions.py:1605,1629``), and the conjunct objects are shared
    between the copies of a state (``constraints.py:56-62``): translating the
    whole set for every query printed and parsed the same conjuncts again and
    again.  Here each conjunct is printed and parsed once, into one long-lived
    IR context (hash-consed: a term shared by two conjuncts is one node), and
    a query only prints the conjuncts it has not seen before, in one
    ``Solver.sexpr()``.  z3 reuses the ids of collected ASTs, so an entry
    keeps its AST alive and an id match is confirmed with ``eq`` (as the
    witness memo does, model.py ``_memo_get``).  The context is dropped and
    rebuilt when it outgrows ``max_nodes`` (lowering adds its rewrites to it)."""

    def __init__(self, max_nodes: int = 1 << 22, max_entries: int = 1 << 18, walk: bool = True):
        self.max_nodes, self.max_entries = max_nodes, max_entries
        self.walk = walk and WALK_ASTS
        self.stats = {"hits": 0, "misses": 0, "prints": 0, "walked": 0, "resets": 0}
        self.reset()

    def reset(self):
        self.ctx = Ctx()
        self.ctx.long_lived = True     # lower_constraints keeps per-conjunct lowerings here
        self.ctx._lowered = {}
        self.entries = {}          # AST id -> (raw, IR node)
        self.decls = {}            # name -> Decl
        self.walker = None
        if self.walk:
            try:
                z3 = _z3()
            except ImportError:
                z3 = None
            from . import z3walk
            if z3 is not None and z3walk.available(z3):
                self.walker = z3walk.Z3Walker(z3, self.ctx)
                self.decls = self.walker.decls     # one table: the walker declares what it meets

    def to_ir(self, raws: Sequence, _retried: bool = False) -> Script:
        if len(self.ctx.nodes) > self.max_nodes or len(self.entries) > self.max_entries:
            self.reset()
            self.stats["resets"] += 1
        ents = [None] * len(raws)
        missing = []
        get = self.entries.get
        for i, r in enumerate(raws):
            e = get(r.get_id())
            if e is not None and (e[0] is r or e[0].eq(r)):
                ents[i] = e
            else:
                missing.append(i)
        self.stats["hits"] += len(raws) - len(missing)
        if missing:
            self.stats["misses"] += len(missing)
            new = [raws[i] for i in missing]
            nodes = None
            if self.walker is not None:
                from .z3walk import SortConflict
                try:
                    nodes = [self.walker.term(r) for r in new]
                    self.stats["walked"] += len(new)
                except SortConflict:
                    # a name this context holds with another sort: once on a fresh
                    # context, then the reference solver
                    if _retried:
                        raise
                    self.reset()
                    self.stats["resets"] += 1
                    return self.to_ir(raws, _retried=True)
                except Unsupported as e:       # the text route below answers (and fails closed itself)
                    log.debug("z3walk: %s; printing the conjuncts instead", e)
            if nodes is None:
                self.stats["prints"] += 1
                sc = parse_script(solver_sexpr(new), self.ctx)
                if len(sc.asserts) != len(new):
                    raise ValueError("z3bridge: the printed script does not hold one assert per conjunct")
                for name, d in sc.decls.items():
                    old = self.decls.get(name)
                    if old is not None and (old.sort != d.sort or old.args != d.args):
                        # one name, two sorts: the shared context cannot hold both.
                        # One retry on a fresh context; a set that conflicts with
                        # itself goes to the reference solver (no loop)
                        if _retried:
                            raise Unsupported(f"z3bridge: '{name}' declared with two sorts in one set")
                        self.reset()
                        self.stats["resets"] += 1
                        return self.to_ir(raws, _retried=True)
                    self.decls[name] = d
                nodes = sc.asserts
            for i, r, n in zip(missing, new, nodes):
                if n.width != BOOL or n.is_array:
                    raise Unsupported("z3bridge: non-Bool assertion")
                ents[i] = self.entries[r.get_id()] = (r, n)
        script = Script(self.ctx)
        script.asserts = [e[1] for e in ents]
        script.decls = self.decls        # every declaration seen (model_from_witness looks names up)
        return script


_cache: Optional[ConjunctCache] = None
CACHE_CONJUNCTS = os.environ.get("MYTHRIL_AMD_CONJUNCT_CACHE", "1") != "0"
WALK_ASTS = os.environ.get("MYTHRIL_AMD_Z3_WALK", "1") != "0"     # z3walk, else print + parse
# a witness z3 confirms only past the pinned budget: "confirm" (default) keeps
# it, with the rest of the query's budget for that second check; "reference"
# hands the query to the reference solver instead, whose own check on the
# unpinned formula may time out there (unknown -> UnsatError, model.py:58-63)
SLOW_RECHECK = os.environ.get("MYTHRIL_AMD_SLOW_RECHECK", "confirm")


def to_ir(raws: Sequence, ctx: Optional[Ctx] = None) -> Script:
    """z3 assertions -> IR: through the process's ConjunctCache (only the
    conjuncts not seen before are printed and parsed), or, given a context or
    with MYTHRIL_AMD_CONJUNCT_CACHE=0, the whole set's text parsed afresh."""
    global _cache
    if ctx is None and CACHE_CONJUNCTS:
        if _cache is None:
            _cache = ConjunctCache()
        return _cache.to_ir(raws)
    return parse_script(solver_sexpr(raws), ctx)


_last = threading.local()     # the last re-check's z3 result ("sat" / "unsat" / "unknown") and time


def last_check() -> dict:
    return getattr(_last, "info", {})


def recheck(raws: Sequence, script: Script, w: Witness, timeout_ms: int, pinned_ms: int) -> Tuple[object, bool]:
    """The z3 re-check of a GPU witness, first under ``pinned_ms`` (with every
    symbol pinned z3 answers at once on almost every query), then, if z3
    answered unknown there, under the query's own ``timeout_ms``.  Returns
    (model or None, slow): ``slow`` marks a witness z3 confirmed only after
    the pinned budget - the queries where the reference's own Optimize.check
    on the unpinned formula may have answered unknown (a timeout, hence
    UnsatError) while the GPU path answers sat (SURVEY.md §7 hard part 5)."""
    m = model_from_witness(raws, script, w, min(timeout_ms, pinned_ms))
    if m is not None or pinned_ms >= timeout_ms or last_check().get("result") != "unknown":
        return m, False
    if SLOW_RECHECK == "reference":
        return None, False      # the reference solver answers the query
    # the second check gets what is left of the query's own budget, so the
    # two z3 calls together stay within it
    m = model_from_witness(raws, script, w, timeout_ms - pinned_ms)
    return m, m is not None


def model_from_witness(raws: Sequence, script: Script, w: Witness, timeout_ms: int = 2000):
    z3 = _z3()
    t0 = time.perf_counter()
    s = z3.Solver()
    s.set(timeout=max(1, int(timeout_ms)))
    s.add(list(raws))
    pins: List = []
    decls = script.decls
    # the witness's own names, looked up in the declarations (which may hold a
    # whole process's symbols: z3bridge.ConjunctCache); Ackermann leaves
    # (cells, applications) are no declarations and are pinned through their
    # array / function below
    for name, fn_vals in w.functions.items():
        d = decls.get(name)
        if d is None or not d.args or not fn_vals:
            continue
        f = z3.Function(name, *[z3.BitVecSort(a.width) for a in d.args], z3.BitVecSort(d.sort.width))
        for args, val in fn_vals.items():
            zargs = [z3.BitVecVal(a, srt.width) for a, srt in zip(args, d.args)]
            pins.append(f(*zargs) == z3.BitVecVal(val, d.sort.width))
    for name, cells in w.arrays.items():
        d = decls.get(name)
        if d is None or d.args or d.sort.kind != "array" or not cells:
            continue
        arr = z3.Array(name, z3.BitVecSort(d.sort.dom), z3.BitVecSort(d.sort.width))
        for idx, val in cells.items():
            pins.append(z3.Select(arr, z3.BitVecVal(idx, d.sort.dom)) == z3.BitVecVal(val, d.sort.width))
    for name, val in w.values.items():
        d = decls.get(name)
        if d is None or d.args or d.sort.kind == "array":
            continue
        if d.sort.kind == "bool":
            pins.append(z3.Bool(name) == z3.BoolVal(bool(val)))
        else:
            pins.append(z3.BitVec(name, d.sort.width) == z3.BitVecVal(val, d.sort.width))
    s.add(pins)
    r = s.check()
    _last.info = {"result": str(r), "ms": (time.perf_counter() - t0) * 1e3}
    if r == z3.sat:
        return s.model()
    log.warning("z3 did not confirm a GPU witness (%s); falling back to the reference solver", r)
    return None
