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
    ap.add_argument("--ab", action="store_true",
                    help="run the profile once per A/B environment (a child process each) and compare")
    a = ap.parse_args()
    if a.ab:
        return ab(a)
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
    from mythril_amd import engine
    engine.PROFILE = {}
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
    phases = {k: {"ms": round(v[0] * 1e3 / n, 5), "calls": round(v[1] / n, 3)} for k, v in engine.PROFILE.items()}
    engine.PROFILE = None
    out = {"queries": n, "hits": hits, "wall_ms_per_query": wall * 1e3 / n,
           "python_ms_per_query": {k: v * 1e3 / n for k, v in py.items()},
           "engine_search_phases_ms_per_query": phases,
           "library_ms_per_query": {k: {"ms": round(ms, 5), "calls": round(c, 3)} for k, ms, c in rows}}
    print(json.dumps(out, indent=1))
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


AB = {
    "base": {},
    "no_witness_thread": {"MYTHRIL_AMD_WITNESS_THREAD": "0"},
    "nt_spin": {"MYTHRIL_AMD_WITNESS_THREAD": "0", "MYTHRIL_AMD_SPIN": "1"},
    "nt_nosdma": {"MYTHRIL_AMD_WITNESS_THREAD": "0", "HSA_ENABLE_SDMA": "0"},
    "nt_spin_nosdma": {"MYTHRIL_AMD_WITNESS_THREAD": "0", "MYTHRIL_AMD_SPIN": "1", "HSA_ENABLE_SDMA": "0"},
}


def ab(a):
    import subprocess
    import tempfile
    res = {}
    for name, env in AB.items():
        with tempfile.NamedTemporaryFile(suffix=".json") as f:
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--every", str(a.every), "--out", f.name],
                               env=dict(os.environ, **env), capture_output=True, text=True, timeout=280)
            if r.returncode != 0:
                print(name, "failed", r.stderr[-2000:], flush=True)
                continue
            d = json.load(open(f.name))
        res[name] = d
        print(f"{name:18s} {d['wall_ms_per_query']:.4f} ms/query  "
              + "  ".join(f"{k} {v['ms']:.4f}" for k, v in d["engine_search_phases_ms_per_query"].items()), flush=True)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
