#!/usr/bin/env python3
"""C3-class preparation through the per-conjunct cache.

The BEC batchTransfer query (tests/golden/solver_log/c3_bec_batchtransfer_overflow.smt2)
is replayed the way LASER sends it: its parent set (every conjunct but the
last) goes through z3bridge.ConjunctCache + prepare() first, then the full
set, whose translation + preparation is timed.  The z3 ASTs are the stand-ins
of tests/fakez3.py (as in tools/replay_latency.py).  Each repetition starts
from a fresh cache; the best and the median of the repetitions are reported
with the phase split of the best one.  The program must be byte-identical to
a whole-set prepare in a fresh context (checked once).

    python tools/c3_prepare.py [--reps 15] [--file NAME] [--out FILE]
"""
import argparse
import gc
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--file", default="c3_bec_batchtransfer_overflow.smt2")
    ap.add_argument("--out", default=None)
    ap.add_argument("--profile", action="store_true", help="cProfile the last repetition's full-set prepare")
    a = ap.parse_args()
    from replay_latency import program_bytes
    from mythril_amd import z3bridge
    from mythril_amd.engine import prepare
    from mythril_amd.smt2 import parse_file, parse_script, to_smt2
    from tests import fakez3
    z = fakez3.module()
    sys.modules["z3"] = z
    z3bridge.solver_sexpr = lambda raws: to_smt2([r.node for r in raws])
    s = parse_file(os.path.join(ROOT, "tests", "golden", "solver_log", a.file))
    text = to_smt2(s.asserts)
    rows = []
    sc = q = None
    for rep in range(a.reps):
        sc = q = None        # the previous repetition's context is freed here, not inside the timed calls
        ws = parse_script(text)         # fresh nodes, fresh stand-in ASTs per repetition
        raws = [z.ast(n) for n in ws.asserts]
        cache = z3bridge.ConjunctCache()
        sp = cache.to_ir(raws[:-1])
        prepare(sp.asserts, sp.ctx)
        tm = {}
        pr = None
        if a.profile and rep == a.reps - 1:
            import cProfile
            pr = cProfile.Profile()
            pr.enable()
        gc.collect()         # the parent's deferred collection (prepare pauses the collector) is not the child's
        t0 = time.perf_counter()
        sc = cache.to_ir(raws)
        t1 = time.perf_counter()
        q = prepare(sc.asserts, sc.ctx, timings=tm)
        t2 = time.perf_counter()
        if pr is not None:
            pr.disable()
            import pstats
            pstats.Stats(pr).sort_stats("cumulative").print_stats(40)
        rows.append({"parse": (t1 - t0) * 1e3, "prepare": (t2 - t1) * 1e3,
                     **{k: v * 1e3 for k, v in tm.items()}})
        if rep == 0:
            fresh = parse_script(text)
            identical = program_bytes(prepare(fresh.asserts, fresh.ctx).program) == program_bytes(q.program)
    best = min(rows, key=lambda r: r["parse"] + r["prepare"])
    out = {"file": a.file, "conjuncts": len(s.asserts), "reps": a.reps, "identical": identical,
           "best_ms": {k: round(v, 3) for k, v in best.items()},
           "median_total_ms": round(statistics.median(r["parse"] + r["prepare"] for r in rows), 3),
           "min_phase_ms": {k: round(min(r[k] for r in rows), 3) for k in best}}
    print(json.dumps(out), flush=True)
    if a.out:
        json.dump({"rows": rows, **out}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
