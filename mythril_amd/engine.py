"""Witness engine: constraint sets -> batched GPU search -> concrete witnesses.

``prepare`` lowers one constraint set (Ackermannisation, width legalisation,
candidate pools) and compiles its search program (verdicts only; the native
compiler, ccompile.py).
``WitnessEngine.search`` launches many programs in one ``mg_search`` call (one
grid row per program, SURVEY.md §8a row A9 batching) and turns each lowest
satisfying index back into a :class:`Witness`: the leaf values come from the
still-loaded search program (``mg_witness_leaves``) when every array index /
function argument is constant, else from a witness program with the same leaf
layout and no conjuncts - only the leaves and every array index / function
argument, traced - compiled on first use.
"""
from __future__ import annotations

import contextlib
import dataclasses
import gc
import logging
import sys
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import isa
from .ccompile import compile_query
from .compiler import LeafSpec, Program, Unsupported
from .ir import BOOL, Ctx, Node, free_vars
from .lower import Lowered, lower_constraints, needs_lowering
from .pools import harvest

log = logging.getLogger(__name__)

DEFAULT_SEED = 0x5EED_0001
DEFAULT_BUDGET = 1 << 22  # candidates per query (early exit + stop-after-hit)
# u32 ops per launch (sum of the programs' ops_per_eval x candidates): bounds what
# a miss costs before z3 answers.  2^22 candidates of a 2 000-op query, a few ms
# on the interpreter; a 14 000-op C3-class query gets ~600 k candidates.
DEFAULT_OP_BUDGET = (1 << 22) * 2000
MIN_CANDIDATES = 1 << 16
# A launch planned at this many u32 ops or more assembles its programs first
# (mythril_amd/asmjit.py: tens of ms per program, 2.5-6x the asm interpreter's
# rate); below it the asm interpreter starts at once.  The default budget's
# launches stay below it: they finish in a few ms.
DEFAULT_ASMJIT_MIN_OPS = 1 << 36


@dataclass
class Witness:
    index: int
    values: Dict[str, int]                           # every scalar leaf (incl. Ackermann leaves)
    arrays: Dict[str, Dict[int, int]] = field(default_factory=dict)
    functions: Dict[str, Dict[Tuple[int, ...], int]] = field(default_factory=dict)


@dataclass
class Query:
    ctx: Ctx
    conjuncts: List[Node]
    lowered: Lowered
    program: Program
    trace_build: "Callable[[], Program]"     # the witness program, compiled on first use
    arg_terms: List[Node]
    arg_chunks: Dict[str, List[List[Node]]] = field(default_factory=dict)
    _trace: Optional[Program] = None
    _trace_future: Optional[object] = None   # a queued compile (_prebuild_witness_programs)
    _long: Optional[Program] = None

    @property
    def long_program(self) -> Program:
        """The program a long search runs (search_phased's launch after the
        probe): ``program`` itself, or the same constraints compiled for the
        asm interpreter's quarter register layout (four waves per SIMD, more
        spills) when that is worth it (_quarter_program).  Same leaf table
        and pools: the same candidates, the same lowest satisfying index."""
        if self._long is None:
            self._long = _quarter_program(self)
        return self._long

    @property
    def trace_program(self) -> Program:
        """The witness program: ``program``'s leaf layout with no conjuncts,
        tracing every leaf and array index / function argument.  Only a
        witness needs it, so it is compiled lazily (or on the host thread
        while the search runs)."""
        if self._trace is None:
            f, self._trace_future = self._trace_future, None
            if f is not None and not f.cancel():
                f.result()           # running or done on the host thread
            if self._trace is None:
                self._trace = self.trace_build()
        return self._trace

    @property
    def ops_per_eval(self) -> int:
        return self.program.ops_per_eval


def prepare(conjuncts: Sequence[Node], ctx: Ctx, use_pools: bool = True,
            timings: Optional[Dict[str, float]] = None) -> Query:
    """Lower, harvest candidate pools and compile one constraint set.
    timings (optional) receives the seconds of each phase (tools/latency_bench.py).
    The cyclic garbage collector is paused for the call: preparation allocates
    thousands of acyclic terms, and a collection pass over the caller's heap
    (a LASER process holds a large one) lands on the query's latency.  Reference
    counting still frees everything; cycles wait for the next pass."""
    was = gc.isenabled()
    gc.disable()
    try:
        return _prepare(conjuncts, ctx, use_pools, timings)
    finally:
        if was:
            gc.enable()


def _prepare(conjuncts, ctx, use_pools, timings) -> Query:
    t0 = time.perf_counter()
    conj = list(conjuncts)
    low = lower_constraints(conj, ctx)
    t1 = time.perf_counter()
    # low.nodes: the topo of the flattened conjuncts, computed once by
    # lower_constraints; harvest collects the var leaves in the same loop
    specs = harvest(low.harvest_conjuncts or low.conjuncts, None, nodes=low.harvest_nodes or low.nodes,
                    memo=ctx.__dict__.setdefault("_harvest", {}) if getattr(ctx, "long_lived", False) else None,
                    split=low.harvest_split) \
        if use_pools else {}
    t2 = time.perf_counter()
    prog = compile_query(low.conjuncts, leaf_specs=specs, reach=(low.flat, low.nodes),
                         memo=ctx.__dict__.setdefault("_records", {}) if getattr(ctx, "long_lived", False) else None)
    if timings is not None:
        timings.update(lower=t1 - t0, pools=t2 - t1, compile=time.perf_counter() - t2)
    # trace every array index / function argument (wider than 256 bits: as 256-bit chunks)
    from .lower import _Rewriter
    chunker = _Rewriter(ctx)
    arg_chunks: Dict[str, List[List[Node]]] = {}
    arg_terms: List[Node] = []
    for al in low.ack.values():
        per = []
        terms = list(al.args) + ([al.value] if al.value is not None else [])
        for a in terms:
            parts = [a] if a.width <= 256 else chunker.chunks(a)
            per.append(parts)
            arg_terms.extend(parts)
        arg_chunks[al.name] = per
    # the search program's leaves lead the trace list in its order, so the witness
    # program numbers them identically: same candidate generator, same values;
    # then the variables only a cell index reads (traced too: the witness
    # carries their values, so the cell and the formula agree)
    have = {n.id for n in prog.leaf_nodes}
    extra = [v for v in _free_vars(arg_terms, ctx) if v.op == "var" and v.id not in have]
    traced = list(prog.leaf_nodes) + extra + arg_terms
    q = Query(ctx, conj, low, prog, lambda: _witness_program(prog, traced), arg_terms)
    q.arg_chunks = arg_chunks
    return q


def _free_vars(terms: List[Node], ctx: Ctx) -> List[Node]:
    """free_vars(terms); in a long-lived context from each term's own list,
    kept per term id and merged by first occurrence (the same list: see
    lower._topo_memo)."""
    if not getattr(ctx, "long_lived", False):
        return free_vars(terms)
    memo = ctx.__dict__.setdefault("_free_vars", {})
    out: Dict[int, Node] = {}
    for t in terms:
        fv = memo.get(t.id)
        if fv is None:
            fv = memo[t.id] = tuple(free_vars([t]))
        for v in fv:
            if v.id not in out:
                out[v.id] = v
    return list(out.values())


# Python-side phase times of WitnessEngine.search (tools/dropin_profile.py):
# a dict to accumulate {phase: [seconds, count]} into, or None (off)
PROFILE: Optional[dict] = None


def _tick(prof: dict, key: str, t0: float) -> float:
    t = time.perf_counter()
    e = prof.get(key)
    if e is None:
        e = prof[key] = [0.0, 0]
    e[0] += t - t0
    e[1] += 1
    return t


_PREBUILD = None   # one host thread for witness-program compiles (_prebuild_witness_programs)
_PREBUILD_LOCK = threading.Lock()


def _build_witness_program(q: "Query") -> None:
    try:
        q._trace = q.trace_build()
    except Exception:   # noqa: BLE001 - trace_program compiles it again and reports the error
        pass
    time.sleep(0)   # hand the GIL back between queries (the search caller waits for it)


# MYTHRIL_AMD_WITNESS_THREAD=1: compile the witness programs on a host thread
# while the search runs (rounds 4-5).  Off by default since round 6: the
# compile is mostly Python, so the thread holds the GIL the searching caller
# needs back after each library call; without it a LASER query costs 0.36
# instead of 0.44 ms on the device path (profiles/r6e, tools/dropin_profile.py
# --ab), and a witness program compiles only when a search found a witness.
import os as _os
WITNESS_THREAD = _os.environ.get("MYTHRIL_AMD_WITNESS_THREAD", "0") == "1"
_os_env = _os.environ.get

# Larger witness programs compile in materialize: their Python part (record
# stream, leaf table) would hold the GIL the returning search call waits for.
PREBUILD_MAX_TERMS = 512


# How soon the caller gets the GIL back from the witness-program thread when
# a program upload or the search returns (sys.setswitchinterval, normally
# 5 ms): the thread holds it through the Python part of a compile, and the
# caller would wait for its forced switch.  Applied only while uploads and a
# search with queued compiles are in flight (_gil_handoff), then restored.
SEARCH_SWITCH_INTERVAL = 2e-5
_HANDOFF = [0, None, None]        # searches in flight, the interval to restore, the one set
_HANDOFF_LOCK = threading.Lock()


@contextlib.contextmanager
def _gil_handoff(active: bool):
    if not active:
        yield
        return
    with _HANDOFF_LOCK:
        if _HANDOFF[0] == 0:
            _HANDOFF[1] = sys.getswitchinterval()
            sys.setswitchinterval(min(_HANDOFF[1], SEARCH_SWITCH_INTERVAL))
            _HANDOFF[2] = sys.getswitchinterval()    # as stored (microseconds)
        _HANDOFF[0] += 1
    try:
        yield
    finally:
        with _HANDOFF_LOCK:
            _HANDOFF[0] -= 1
            # restored only if nobody else changed it meanwhile
            if _HANDOFF[0] == 0 and sys.getswitchinterval() == _HANDOFF[2]:
                sys.setswitchinterval(_HANDOFF[1])


# A stop-after-hit search first tries the lowest PROBE_CANDIDATES indices in a
# launch of their own: most satisfiable LASER queries have a witness there
# (pool-first candidate order), and the full launch runs every block's first
# chunk (2 048 blocks x 256 candidates) before any can stop.  Programs with no
# witness in the probe continue from its end; the lowest satisfying index is
# the same either way.
PROBE_CANDIDATES = 1 << 16


def search_phased(dev, dps, seed: int, begin: int, count: int, flags: int, long_programs=None):
    """dev.search(dps, seed, begin, count, flags) with the probe launch above
    (stop-after-hit searches longer than twice the probe); the statistics of
    both launches summed.  long_programs: per program, a callable of the
    candidates left giving the program the launch after the probe runs
    instead (search_program: the same candidates; loaded here and freed
    after that launch)."""
    if not (flags & isa.FLAG_STOP_AFTER_HIT) or count <= 2 * PROBE_CANDIDATES:
        return dev.search(dps, seed, begin, count, flags)
    found, st = dev.search(dps, seed, begin, PROBE_CANDIDATES, flags)
    rest = [i for i, f in enumerate(found) if f is None]
    if rest:
        rdps, extra = [], []
        try:
            for i in rest:
                # a program with an assembled kernel attached keeps it (ADVICE r5:
                # the long program would run on the interpreter instead)
                lp = long_programs[i](count - PROBE_CANDIDATES) \
                    if long_programs is not None and not getattr(dps[i], "assembled", None) else None
                if lp is not None and lp is not dps[i].prog:
                    d = dev.load(lp)
                    extra.append(d)
                    # the recompile is for the asm interpreter; on any other
                    # engine it is only longer (engine_of is the loader's choice)
                    rdps.append(d if not hasattr(dev, "engine_of") or dev.engine_of(d) == "asm" else dps[i])
                else:
                    rdps.append(dps[i])
            f2, st2 = dev.search(rdps, seed, begin + PROBE_CANDIDATES, count - PROBE_CANDIDATES, flags)
        finally:
            for d in extra:
                d.free()
        found = list(found)
        for i, f in zip(rest, f2):
            found[i] = f
        st = {k: (v + st2[k] if isinstance(v, (int, float)) and k in st2 else v) for k, v in st.items()}
    return found, st


# MYTHRIL_AMD_WITNESS_IN_LAUNCH=0: read witnesses with a launch of their own
# after the search (mg_eval_program) instead of in the search's synchronisation
WITNESS_IN_LAUNCH = _os_env("MYTHRIL_AMD_WITNESS_IN_LAUNCH", "1") != "0"


def search_with_witnesses(dev, dps, queries, seed: int, begin: int, count: int, flags: int, long_programs=None):
    """search_phased, with each query's witness read in the search's own
    synchronisation: the search is enqueued
    (mg_search_begin), the witness programs compile on the host while the
    device searches, and mg_search_end evaluates each at the index its search
    found, queued after the search, one synchronisation for all of it.
    Returns (found, stats, traces): traces[i] is query i's witness trace
    column, or None (no witness; or the caller evaluates it)."""
    n = len(dps)
    probe = bool(flags & isa.FLAG_STOP_AFTER_HIT) and count > 2 * PROBE_CANDIDATES
    first = PROBE_CANDIDATES if probe else count
    dev.search_begin(dps, seed, begin, first, flags)
    wps = None
    try:
        wps = [q.trace_program for q in queries]
        # only a witness program with the search program's leaf layout reads
        # the same candidate (else materialize refuses it: z3 answers)
        wps = [p if _same_leaves(q, p) else None for q, p in zip(queries, wps)]
    finally:
        if wps is None:          # the compile raised: complete the search, then re-raise
            dev.search_end(None)
    found, st, traces = dev.search_end(wps)
    rest = [i for i, f in enumerate(found) if f is None]
    if not probe or not rest:
        return found, st, traces
    rdps, extra = [], []
    try:
        for i in rest:
            lp = long_programs[i](count - PROBE_CANDIDATES) \
                if long_programs is not None and not getattr(dps[i], "assembled", None) else None
            if lp is not None and lp is not dps[i].prog:
                d = dev.load(lp)
                extra.append(d)
                rdps.append(d if not hasattr(dev, "engine_of") or dev.engine_of(d) == "asm" else dps[i])
            else:
                rdps.append(dps[i])
        dev.search_begin(rdps, seed, begin + PROBE_CANDIDATES, count - PROBE_CANDIDATES, flags)
        f2, st2, t2 = dev.search_end([wps[i] for i in rest])
    finally:
        for d in extra:
            d.free()
    found, traces = list(found), list(traces)
    for k, i in enumerate(rest):
        found[i], traces[i] = f2[k], t2[k]
    st = {k: (v + st2[k] if isinstance(v, (int, float)) and k in st2 else v) for k, v in st.items()}
    return found, st, traces


def _same_leaves(q: "Query", p: Program) -> bool:
    """The witness program p draws the search program's leaves in its order
    (compile_trace_native shares the leaf table itself; a fresh compile must
    lead with the same names)."""
    return p.leaves is q.program.leaves or \
        [n.name for n in p.leaf_nodes[:len(q.program.leaf_nodes)]] == [n.name for n in q.program.leaf_nodes]


def _prebuild_witness_programs(queries) -> bool:
    """Queue the witness programs a search may need on a host thread, which
    compiles them while the device searches (the search call releases the
    GIL): those of queries whose cells have a non-constant index (the rest
    read their leaves from the search program, mg_witness_leaves).
    Query.trace_program takes a finished one, waits for a running one and
    compiles a not yet started one itself, so nothing is compiled twice and
    no search waits for the compiles of queries that found nothing."""
    if not WITNESS_THREAD:
        return False
    todo = [q for q in queries if q._trace is None and q._trace_future is None
            and len(q.arg_terms) <= PREBUILD_MAX_TERMS and not all(t.op == "const" for t in q.arg_terms)]
    if not todo:
        return False
    global _PREBUILD
    if _PREBUILD is None:
        with _PREBUILD_LOCK:
            if _PREBUILD is None:
                from concurrent.futures import ThreadPoolExecutor
                _PREBUILD = ThreadPoolExecutor(max_workers=1, thread_name_prefix="mw-witness-program")
    for q in todo:
        q._trace_future = _PREBUILD.submit(_build_witness_program, q)
    return True


# The asm interpreter's quarter register layout (mw_kernels.hip
# mw_search_asm_kernel_q, asmgen.py variant("quarter")): 5 W and 16 N slots,
# four waves per SIMD where the other layouts run three or two; its LDS
# budget per thread (spill words and pool rows) is QUARTER_LDS_WORDS.  A
# program the compiler allocated over more slots is compiled again within
# those for long searches, when it spills within that budget and grows by at
# most QUARTER_MAX_GROWTH in instructions (profiles/r5c: the quarter kernel
# runs the LASER group 1.28x as fast as the narrow and wide ones).
QUARTER_SLOTS = (5, 16)
NARROW_SLOTS = (8, 24)      # the narrow layout's files (asmgen.py variant "narrow")
# ... and only when the search left is long enough to repay that compile
# (~0.3 ms host, the quarter kernel ~25 % faster): candidates x instructions
# at least this (profiles/r5f: for a 2^22-candidate LASER miss, 0.32 ms of
# kernel, the recompile cost more than it saved)
LONG_PROGRAM_MIN_WORK = 1 << 31
QUARTER_LDS_WORDS = isa.ASM_LDS_WORDS["quarter"]
QUARTER_MAX_GROWTH = 1.3
NARROW_MAX_GLOBAL_SPILL = 8


def _slots_used(p: Program) -> Tuple[int, int]:
    """(W slots, N slots) the program's results occupy (highest + 1)."""
    mw = mn = -1
    code = p.code
    for i in range(1, len(code), 4):
        w, n = isa.decode_dst(int(code[i]) & 0xFFFF)
        if w is not None and w > mw:
            mw = w
        if n is not None and n > mn:
            mn = n
    return mw + 1, mn + 1


def _pool_rows(p: Program) -> int:
    """LDS words per thread the program's pool takes (256 threads a block)"""
    return (int(p.pool.size) + 255) // 256 if p.pool is not None else 0


def _lands_on(p: Program, layout: str) -> bool:
    """Whether the loader (mw_prog_load) puts p on the asm kernel of this
    register layout: its narrow constants fit the layout's constant
    registers, and its pool (the quarter layout: its spill words too) fits
    the layout's LDS budget.  Register files are the compile's own slots."""
    if len(isa.asm_narrow_constants(p.code, p.consts)) > isa.ASM_NK_BY_LAYOUT[layout]:
        return False
    rows = _pool_rows(p)
    if layout == "quarter":
        return p.n_spill + rows <= isa.ASM_LDS_WORDS["quarter"]
    return rows <= isa.ASM_LDS_WORDS[layout]


def _global_spill(p: Program, layout: str) -> int:
    """Spill words per thread that fall outside the layout's LDS budget (the global spill buffer)."""
    return max(0, p.n_spill + _pool_rows(p) - isa.ASM_LDS_WORDS[layout])


def _quarter_program(q: "Query") -> Program:
    """q.long_program's compile: only programs the asm
    interpreter runs are recompiled, only into layouts whose switch is on,
    and a recompiled program is kept only if the loader will put it on the
    kernel it was compiled for (_lands_on) - otherwise it would run with more
    instructions on a wider kernel or the compiled interpreter, a pure loss."""
    p = q.program
    sw = isa.asm_switches()
    if not sw["narrow"] or not isa.asm_eligible(p.code, p.leaves, p.consts):
        return p
    w, n = _slots_used(p)
    if (w <= QUARTER_SLOTS[0] and n <= QUARTER_SLOTS[1]) or _pool_rows(p) >= QUARTER_LDS_WORDS:
        return p       # fits already (the loader picks the quarter kernel), or its pool alone fills the budget
    fixed = {s.name: dataclasses.replace(s, pool=None if s.pool is None else list(s.pool)) for s in p.leaf_specs}
    if not sw["quarter"]:
        return _narrow_program(q, fixed)
    try:
        qp = compile_query(q.lowered.conjuncts, leaf_specs=fixed, reach=(q.lowered.flat, q.lowered.nodes),
                           slots=QUARTER_SLOTS)
    except Exception:   # noqa: BLE001 - the program as it is
        return p
    if (qp.n_insn > QUARTER_MAX_GROWTH * p.n_insn or not _lands_on(qp, "quarter")
            or not isa.asm_eligible(qp.code, qp.leaves, qp.consts)
            or not np.array_equal(qp.leaves, p.leaves) or not np.array_equal(qp.pool, p.pool)):
        return _narrow_program(q, fixed)
    return qp


def _narrow_program(q: "Query", fixed) -> Program:
    """A wide-layout program recompiled into the narrow layout's 24 N slots
    (three waves per SIMD instead of two) when that costs at most
    QUARTER_MAX_GROWTH in instructions (C3 with grids: 35 N slots -> 24,
    460 -> 480 instructions), lands on the narrow kernel, and puts at most
    NARROW_MAX_GLOBAL_SPILL more spill words in global memory than the
    original does on the wide one (C3: 6 words past the 52-word budget, and
    still 1.27x as fast, profiles/r5zd)."""
    p = q.program
    w, n = _slots_used(p)
    if w <= NARROW_SLOTS[0] and n <= NARROW_SLOTS[1]:
        return p
    try:
        np_ = compile_query(q.lowered.conjuncts, leaf_specs=fixed, reach=(q.lowered.flat, q.lowered.nodes),
                            slots=NARROW_SLOTS)
    except Exception:   # noqa: BLE001 - the program as it is
        return p
    if (np_.n_insn > QUARTER_MAX_GROWTH * p.n_insn or not _lands_on(np_, "narrow")
            or not isa.asm_eligible(np_.code, np_.leaves, np_.consts)
            or _global_spill(np_, "narrow") > _global_spill(p, "wide") + NARROW_MAX_GLOBAL_SPILL
            or not np.array_equal(np_.leaves, p.leaves) or not np.array_equal(np_.pool, p.pool)):
        return p
    return np_


def search_program(q: "Query", candidates: int) -> Program:
    """The program a search of `candidates` candidates runs: q.long_program
    when the work repays its compile (LONG_PROGRAM_MIN_WORK), else q.program."""
    if candidates * max(1, q.program.n_insn) >= LONG_PROGRAM_MIN_WORK:
        return q.long_program
    return q.program


def _witness_program(prog: Program, traced: List[Node]) -> Program:
    """The witness program of `prog`: its leaf layout (pool fields already
    assigned; copies, layout_leaves updates the specs it is given), no
    conjuncts, the leaves and cell indices traced.  A natively compiled prog
    gives it from its own record stream and leaf table
    (ccompile.compile_trace_native: the same program, without a second
    serialisation and layout)."""
    from .ccompile import compile_trace_native
    wp = compile_trace_native(prog, traced)
    if wp is not None:
        return wp
    fixed = {s.name: dataclasses.replace(s, pool=None if s.pool is None else list(s.pool))
             for s in prog.leaf_specs}
    return compile_query([], leaf_specs=fixed, trace=traced)


def _combine_chunks(values: Dict[str, int], name: str, width: int) -> int:
    if name in values:
        return values[name]
    v, lo, k = 0, 0, 0
    while lo < width:
        v |= values.get(f"{name}#{k}", 0) << lo
        lo += 256
        k += 1
    return v


class WitnessEngine:
    """Owns one device context; everything goes through the C-ABI.

    The witnesses ``search`` returns are NOT re-evaluated on the device by
    default: the search launch found their index satisfying, and their
    values come from the leaf generator (or a witness program) at that
    index.  The drop-in re-checks every witness with z3 before it is used
    (model.py, z3bridge.model_from_witness) and the tests with the oracle;
    other callers that want a device-side check pass ``verify=True`` (one
    mg_eval_generated of the search program at the index per witness; a
    witness it does not confirm is dropped and counted in
    ``stats["verify_rejects"]``)."""

    def __init__(self, device: int = 0, seed: int = DEFAULT_SEED, budget: int = DEFAULT_BUDGET, dev=None,
                 op_budget: Optional[int] = DEFAULT_OP_BUDGET, asmjit_min_ops: Optional[int] = DEFAULT_ASMJIT_MIN_OPS,
                 verify: bool = False):
        if dev is None:
            from .runtime import Device  # raises EngineUnavailable without the HIP library / GPU
            dev = Device(device)
        self.dev = dev
        self.seed = seed
        self.budget = budget
        self.op_budget = op_budget
        self.asmjit_min_ops = asmjit_min_ops   # None / 0: never assemble
        self.verify = verify
        self.stats = {"searches": 0, "programs": 0, "hits": 0, "evals": 0, "kernel_ms": 0.0, "assembled": 0,
                      "assemble_s": 0.0}

    def close(self):
        self.dev.close()

    def search(self, queries: Sequence[Query], count: Optional[int] = None, begin: int = 0,
               flags: int = isa.FLAG_EARLY_EXIT | isa.FLAG_STOP_AFTER_HIT) -> List[Optional[Witness]]:
        if not queries:
            return []
        count = count or self.launch_count(queries)
        dps = []
        hits = set()
        prof = PROFILE
        t0 = time.perf_counter() if prof is not None else 0.0
        # the witness programs compile on a host thread while the programs
        # upload and the device searches (those calls release the GIL): a
        # witness then costs one upload and one launch (materialize)
        queued = _prebuild_witness_programs(queries)
        try:
            with _gil_handoff(queued):
                if prof is not None:
                    _tick(prof, "prebuild", t0)
                for q in queries:   # a failed load frees the programs already loaded
                    dps.append(self.dev.load(q.program))
                if prof is not None:
                    t0 = _tick(prof, "load", t0)
                if (self.asmjit_min_ops and hasattr(self.dev, "attach_asm")
                        and count * sum(q.ops_per_eval for q in queries) >= self.asmjit_min_ops):
                    self._assemble(dps)
                longs = [lambda n, q=q: search_program(q, n) for q in queries]
                traces = [None] * len(queries)
                if WITNESS_IN_LAUNCH and not queued and hasattr(self.dev, "search_begin"):
                    found, st, traces = search_with_witnesses(self.dev, dps, queries, self.seed, begin, count, flags,
                                                              longs)
                else:
                    found, st = search_phased(self.dev, dps, self.seed, begin, count, flags, longs)
                if prof is not None:
                    t0 = _tick(prof, "search", t0)
            self.stats["searches"] += 1
            self.stats["programs"] += len(queries)
            self.stats["evals"] += st["evals"]
            self.stats["kernel_ms"] += st["kernel_ms"]
            out: List[Optional[Witness]] = []
            for q, dp, idx, tr in zip(queries, dps, found, traces):
                if idx is None:
                    w = None
                elif tr is not None:     # read in the search's synchronisation
                    w = self._decode_trace(q, q.trace_program, idx, tr)
                else:
                    w = self.materialize(q, idx, dp)
                if w is not None and self.verify:
                    v, _ = self.dev.eval_generated(dp, self.seed, idx, 1, trace=False)
                    if not int(v[0]):
                        log.warning("witness engine: the search program does not hold at index %d", idx)
                        self.stats["verify_rejects"] = self.stats.get("verify_rejects", 0) + 1
                        w = None
                if w is not None:
                    self.stats["hits"] += 1
                    hits.add(id(q))
                out.append(w)
            if prof is not None:
                t0 = _tick(prof, "materialize", t0)
        finally:
            for dp in dps:
                dp.free()
            if queued:
                # the queued compiles of queries without a witness (all of them
                # when the search raised) are withdrawn: they would hold the GIL
                # against the caller's next prepare() and keep the queries alive,
                # and a later search's compiles would queue behind them
                for q in queries:
                    f = q._trace_future
                    if f is not None and id(q) not in hits:
                        f.cancel()
                        q._trace_future = None
            if prof is not None:
                _tick(prof, "free", t0)
        return out

    def _assemble(self, dps) -> None:
        """Attach assembled kernels to the eligible programs (parallel
        llvm-mc runs; on-disk cache).  Any failure leaves that program on the
        asm interpreter: same results, only slower."""
        import time
        from concurrent.futures import ThreadPoolExecutor

        from . import asmjit
        if not asmjit.available():
            return
        todo = [dp for dp in dps if asmjit.eligible(dp.prog)]
        t0 = time.perf_counter()
        with ThreadPoolExecutor(max(1, min(8, len(todo)))) as ex:
            futs = [(dp, ex.submit(asmjit.assemble, dp.prog)) for dp in todo]
            for dp, f in futs:
                try:
                    image, name, _ = f.result()
                    self.dev.attach_asm(dp, image, name)
                    self.stats["assembled"] += 1
                except Exception as e:   # noqa: BLE001 - stays on the interpreter
                    log.warning("assembled kernel unavailable for %s: %s", getattr(dp.prog, "n_insn", "?"), e)
        self.stats["assemble_s"] += time.perf_counter() - t0

    def launch_count(self, queries: Sequence[Query]) -> int:
        """Candidates per query for one launch: the candidate budget, cut so the
        launch stays within op_budget u32 ops (never below MIN_CANDIDATES)."""
        if not self.op_budget:
            return self.budget
        ops = max(1, sum(q.ops_per_eval for q in queries))
        return max(min(self.budget, MIN_CANDIDATES), min(self.budget, self.op_budget // ops))

    def materialize(self, q: Query, index: int, search_dp=None) -> Optional[Witness]:
        """The witness at candidate ``index``.  When every array index and
        function argument is a constant (each such cell is then a leaf of its
        own), the leaf values are all of it: one mg_witness_leaves launch on
        the still-loaded search program.  Otherwise the values are read from
        the witness program (leaves plus the traced argument terms), one
        mg_eval_generated launch.  Neither re-evaluates the verdict on the
        device: the search launch found the index satisfying, and every
        witness is re-checked against the original constraints before it is
        used (z3 in the drop-in, model.py / z3bridge.model_from_witness; the
        oracle in the tests)."""
        if (search_dp is not None and getattr(self.dev, "witness_leaves", None) is not None
                and all(t.op == "const" for t in q.arg_terms)):
            return self._from_leaves(q, index, self.dev.witness_leaves(search_dp, self.seed, index))
        return self._materialize_traced(q, index, search_dp)

    def _from_leaves(self, q: Query, index: int, leaf_values) -> Witness:
        values = {n.name: v for n, v in zip(q.program.leaf_nodes, leaf_values)}
        w = Witness(index, values)
        self._ack_cells(q, w, values, lambda t: t.val)
        return w

    @staticmethod
    def _ack_cells(q: Query, w: Witness, values: Dict[str, int], term_value) -> None:
        arrays, functions, chunks = w.arrays, w.functions, q.arg_chunks
        for al in q.lowered.ack.values():
            args = []
            for parts in chunks[al.name]:
                if len(parts) == 1:
                    args.append(term_value(parts[0]))
                    continue
                v = 0
                for k, t in enumerate(parts):
                    v |= term_value(t) << (256 * k)
                args.append(v)
            if al.value is not None:
                val = args.pop()  # defined value (keccak inverse = hashed input)
            else:
                val = values.get(al.name)
                if val is None:
                    val = _combine_chunks(values, al.name, al.width)
            if al.kind == "select":
                cells = arrays.get(al.base)
                if cells is None:
                    cells = arrays[al.base] = {}
                cells[args[0]] = val
            else:
                cells = functions.get(al.base)
                if cells is None:
                    cells = functions[al.base] = {}
                cells[tuple(args)] = val

    def _materialize_traced(self, q: Query, index: int, search_dp=None) -> Optional[Witness]:
        from .runtime import EngineError, trace_column
        t0 = time.perf_counter()
        waited = q._trace is None
        p = q.trace_program
        if PROFILE is not None:
            _tick(PROFILE, "materialize/witness program" + (" (waited)" if waited else ""), t0)
        # a witness program built from the search program's stream shares its
        # leaf table (compile_trace_native checked the leaf order).  Otherwise
        # the search program's leaves must lead the witness program's in the
        # same order; it may have more: variables only a cell index reads and
        # no conjunct (a DependencyPruner tuple `f(x) == 1` reads no x), whose
        # values no verdict depends on
        if not _same_leaves(q, p):
            # an EngineError, so get_model's handler sends the query to z3
            raise EngineError("witness program's leaf layout differs from the search program's")
        t1 = time.perf_counter()
        if hasattr(self.dev, "eval_program"):
            # upload, evaluation and release in one library call (mg_eval_program)
            t2 = t1
            _, trace = self.dev.eval_program(p, self.seed, index, 1)
        else:
            dp = self.dev.load(p)
            t2 = time.perf_counter()
            try:
                _, trace = self.dev.eval_generated(dp, self.seed, index, 1)
            finally:
                dp.free()
        t3 = time.perf_counter()
        # seconds per step of the last traced witness (tools/latency_bench.py)
        self.last_materialize = {"program": t1 - t0, "load": t2 - t1, "eval": t3 - t2}
        if PROFILE is not None:
            PROFILE.setdefault("materialize/load (mg_prog_load)", [0.0, 0])[0] += t2 - t1
            PROFILE.setdefault("materialize/eval (mg_eval_generated)", [0.0, 0])[0] += t3 - t2
        return self._decode_trace(q, p, index, trace)

    def _decode_trace(self, q: Query, p: Program, index: int, trace) -> Witness:
        """The witness from the witness program p's trace column at index."""
        from .runtime import trace_column
        col = trace_column(trace)   # the one candidate's rows, read per node below
        tmap, frm = p.trace_map, int.from_bytes
        values = {}
        for n in p.leaf_nodes:      # unpack_one, inlined
            row, cls = tmap[n.id]
            values[n.name] = frm(col[4 * row:4 * row + (32 if cls == "W" else 4)], "little")
        w = Witness(index, values)

        def term_value(t):   # unpack_one, inlined: one call per traced term
            if t.op == "const":
                return t.val
            row, cls = tmap[t.id]
            return frm(col[4 * row:4 * row + (32 if cls == "W" else 4)], "little")
        self._ack_cells(q, w, values, term_value)
        return w
