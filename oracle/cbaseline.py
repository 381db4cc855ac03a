"""ORACLE (test infrastructure only): bench.py's cpu_baseline leg.

Times the CPU restatement evaluating the same C5 program on the same
candidate indices the GPU searches (index 0, 1, 2, ...), bounded by a wall
budget.  Uses the C restatement (oracle/c, OpenMP over all host cores) when
built, else the pure-Python oracle on one core.  kind = "port": the reference
path (z3 substitute+simplify) is not installed here or on the GPU box
(SURVEY.md §0), so the baseline is our restatement of its semantics.
"""
from __future__ import annotations

import os
import time


def run(syn, prog, budget_s: float = 10.0, verdicts: bool = False):
    """The baseline record; with verdicts=True also the verdict vector of the
    evaluated indices 0..n-1 (C restatement only; None from the Python path)."""
    try:
        from . import cdag
        if cdag.available():
            return cdag.baseline(syn, prog, budget_s, verdicts=verdicts)
    except Exception:  # pragma: no cover - fall through to Python
        pass
    if verdicts:
        return run(syn, prog, budget_s), None
    from .dag_eval import eval_nodes
    from .philox import random_leaf
    import zlib

    names = [n.name for n in prog.leaf_nodes]
    salts = [zlib.crc32(nm.encode()) & 0xFFFFFFFF for nm in names]
    n = 0
    sat = 0
    t0 = time.perf_counter()
    while True:
        m = {nm: random_leaf(syn.seed, s, n, 256) for nm, s in zip(names, salts)}
        vals = eval_nodes(syn.conjuncts, m)
        sat += int(all(vals[c.id] for c in syn.conjuncts))
        n += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "evals/s", "cores": 1, "kind": "port",
            "sample": f"{n} candidates (indices 0..{n - 1}) of the same C5 program, pure-Python oracle, "
                      f"{dt:.1f} s", "satisfied": sat}
