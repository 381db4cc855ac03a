#!/usr/bin/env python3
"""Where a drop-in query's device time goes, inside the library (VERDICT r5
item 3): the LASER corpus searched as WitnessEngine.search does, with the
library's per-step wall times on (MYTHRIL_AMD_STEP_TIMES=1, mw_inflight.h),
and the Python side of each call timed around it.  Prints the mean ms per
query of every "call/step" and of the Python wrappers.

    python tools/dropin_profile.py [--every K] [--out FILE]
"""
import argparse
import glob
import json
import os
import sys
import time

os.environ.setdefault("MYTHRIL_AMD_STEP_TIMES", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--every", type=int, default=2, help="profile every K-th query of the corpus")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from mythril_amd import runtime
    from mythril_amd.engine import WitnessEngine, prepare
    from mythril_amd.smt2 import parse_file
    files = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", "laser", "*.smt2.gz")))[::a.every]
    qs = []
    for f in files:
        s = parse_file(f)
        qs.append(prepare(s.asserts, s.ctx))
    eng = WitnessEngine(device=0)
    for q in qs[:8]:      # warm-up: pools, pinned buffers, code paths
        eng.search([q])
    runtime.step_times()
    py = {"engine.search": 0.0}
    t0 = time.perf_counter()
    hits = 0
    for q in qs:
        t = time.perf_counter()
        w = eng.search([q])[0]
        py["engine.search"] += time.perf_counter() - t
        hits += w is not None
    wall = time.perf_counter() - t0
    lib = runtime.step_times()
    n = len(qs)
    rows = sorted(((k, ms / n, c / n) for k, (ms, c) in lib.items()), key=lambda r: -r[1])
    out = {"queries": n, "hits": hits, "wall_ms_per_query": wall * 1e3 / n,
           "python_ms_per_query": {k: v * 1e3 / n for k, v in py.items()},
           "library_ms_per_query": {k: {"ms": round(ms, 5), "calls": round(c, 3)} for k, ms, c in rows}}
    print(json.dumps(out, indent=1))
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
