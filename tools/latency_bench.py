#!/usr/bin/env python3
"""Per-query latency of the drop-in path: what one
get_model(...) feasibility query costs before z3 would be asked.

For every query of the committed corpora (tests/golden/solver_log: the C2-C4
shapes; tests/golden/laser: LASER-shaped queries over the reference's own
bytecode) it reports, in ms:
  parse      SMT-LIB2 text -> IR (stands in for z3bridge.to_ir; no z3 here)
  lower      Ackermannisation, congruence, wide legalisation (lower.py)
  pools      candidate pools / domains (pools.py)
  compile    bytecode + register allocation (compiler.py)
  search     one mg_search launch, early exit + stop-after-hit, the engine's
             default per-query budget (device; wall time of the call)
  materialise  the witness values of the found index with the search program
             still loaded (only on a witness): one mg_witness_leaves launch when
             every array index / function argument is constant, else one
             launch of the witness program (compiled on a host thread during
             the search, as WitnessEngine.search does)
and the medians per corpus.  Without a GPU (--no-device) only the host
phases are timed.

    python tools/latency_bench.py [--out FILE] [--no-device]
"""
import argparse
import glob
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-device", action="store_true")
    a = ap.parse_args()
    from mythril_amd.engine import (WitnessEngine, _gil_handoff, _prebuild_witness_programs, prepare,
                                     search_phased, search_program)
    from mythril_amd import engine as engine_mod
    from mythril_amd.smt2 import parse_file
    eng = None if a.no_device else WitnessEngine(device=0)
    calls = []    # every mg_search of the current query: (call wall, library wall, kernel) ms
    if eng is not None:
        real_search = eng.dev.search

        def timed_search(*args, **kw):
            t = time.perf_counter()
            res = real_search(*args, **kw)
            calls.append(((time.perf_counter() - t) * 1e3, res[1].get("wall_ms", 0.0), res[1].get("kernel_ms", 0.0)))
            return res
        eng.dev.search = timed_search
    rows = []
    for corpus in ("solver_log", "laser"):
        files = sorted(glob.glob(os.path.join(ROOT, "tests", "golden", corpus, "*.smt2*")))
        for f in files:
            t0 = time.perf_counter()
            s = parse_file(f)
            t_parse = time.perf_counter() - t0
            tm = {}
            q = prepare(s.asserts, s.ctx, timings=tm)
            row = {"corpus": corpus, "file": os.path.basename(f), "conjuncts": q.program.n_conjuncts,
                   "insns": q.program.n_insn, "parse": t_parse * 1e3,
                   **{k: v * 1e3 for k, v in tm.items()}}
            row["prepare"] = row["lower"] + row["pools"] + row["compile"]
            if eng is not None:
                t1 = time.perf_counter()
                # as WitnessEngine.search: the witness program compiles on the
                # host thread while the program uploads and the device searches
                queued = _prebuild_witness_programs([q])
                t_q = time.perf_counter()
                with _gil_handoff(queued):
                    dp = eng.dev.load(q.program)
                t_l = time.perf_counter()
                calls.clear()
                try:
                    tr = None
                    with _gil_handoff(queued):
                        # as WitnessEngine.search: the launch after the probe runs
                        # the query's long program (the quarter layout's compile);
                        # since round 6 the witness program compiles while the
                        # device searches and is evaluated in the search's own
                        # synchronisation (engine.search_with_witnesses)
                        longs = [lambda n: search_program(q, n)]
                        if engine_mod.WITNESS_IN_LAUNCH and not queued:
                            (idx,), st, (tr,) = engine_mod.search_with_witnesses(
                                eng.dev, [dp], [q], eng.seed, 0, eng.launch_count([q]), 3, longs)
                        else:
                            (idx,), st = search_phased(eng.dev, [dp], eng.seed, 0, eng.launch_count([q]), 3, longs)
                    row["search"] = (time.perf_counter() - t1) * 1e3
                    row["kernel"] = st["kernel_ms"]
                    # where the search's time goes: queueing the witness compile,
                    # the upload call, and per mg_search call its Python/ctypes
                    # wall, the library's own wall and the kernel time
                    row["search_parts"] = {"prebuild": (t_q - t1) * 1e3, "load": (t_l - t_q) * 1e3,
                                           "calls": [[round(x, 4) for x in c] for c in calls]}
                    if idx is not None:
                        # as WitnessEngine.search does: the search program is still
                        # loaded (mg_witness_leaves when every cell index is constant)
                        t2 = time.perf_counter()
                        eng.last_materialize = None
                        if tr is not None:     # the trace came back with the search: decode only
                            eng._decode_trace(q, q.trace_program, idx, tr)
                        else:
                            eng.materialize(q, idx, dp)
                        row["materialise"] = (time.perf_counter() - t2) * 1e3
                        if getattr(eng, "last_materialize", None):
                            row["materialise_parts"] = {k: v * 1e3 for k, v in eng.last_materialize.items()}
                        row["leaf_path"] = all(t.op == "const" for t in q.arg_terms)
                finally:
                    dp.free()
                row["witness"] = idx is not None
            rows.append(row)
            print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in row.items()}), flush=True)
    summary = {}
    for corpus in ("solver_log", "laser"):
        rs = [r for r in rows if r["corpus"] == corpus]
        summary[corpus] = {k: statistics.median(r[k] for r in rs if k in r)
                           for k in ("parse", "lower", "pools", "compile", "prepare", "search", "kernel", "materialise")
                           if any(k in r for r in rs)}
        summary[corpus]["queries"] = len(rs)
    print(json.dumps({"median_ms": summary}), flush=True)
    if a.out:
        json.dump({"rows": rows, "median_ms": summary}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
