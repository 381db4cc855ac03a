#!/usr/bin/env python3
"""Host cost of the drop-in's translation + preparation in LASER's query order
(VERDICT r4 item 2): the whole-set path against the per-conjunct cache.

Every scenario of tools/make_laser_corpus.py is recorded by the concolic LASER
restatement (tests/laser_concolic.py) and its get_model queries are replayed
in the order LASER issues them (the recorded order), as one Mythril run per
scenario.  A query's conjuncts are stand-in z3 ASTs: one object per distinct
term, shared by every set that holds it, as LASER's Constraints copies share
their Bool objects (constraints.py:56-62).  z3's ``Solver.sexpr()`` is stood
in for by our printer (mythril_amd/smt2.py to_smt2, the same text shape) and
is NOT timed: z3 is absent here and on the GPU box.

  whole   parse_script of the whole set's text (what z3bridge.to_ir did
          through round 4), then prepare() in the fresh context
  cached  z3bridge.ConjunctCache.to_ir (only unseen conjuncts translated, by
          the z3 AST walker mythril_amd/z3walk.py over tests/fakez3.py's
          stand-in ASTs, into the run's long-lived context), then prepare()
          (per-conjunct lowering, congruence pairs and harvest contributions
          reused).  --print: unseen conjuncts printed and parsed instead.
The stand-in ASTs cost a Python attribute read where z3py makes a ctypes
call (decl(), kind(), children()): the walker's time on real z3 is higher.

Programs must be byte-identical between the two paths (checked per query).

    python tools/replay_latency.py [--out FILE] [--only SUBSTR]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def program_bytes(p) -> bytes:
    import numpy as np
    parts = [np.asarray(p.code, dtype=np.uint32).tobytes(), np.asarray(p.consts, dtype=np.uint32).tobytes(),
             np.asarray(p.leaves, dtype=np.uint32).tobytes(),
             np.asarray(getattr(p, "pools", []), dtype=np.uint32).tobytes()]
    return b"|".join(parts) + repr((p.ops_per_eval, p.n_spill if hasattr(p, "n_spill") else 0)).encode()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", default=None)
    ap.add_argument("--no-check", action="store_true", help="skip the byte-identity check")
    ap.add_argument("--print", action="store_true", help="cached route prints + parses unseen conjuncts")
    a = ap.parse_args()
    from make_laser_corpus import SCENARIOS, load_code, scenario_balances
    from mythril_amd import z3bridge
    from mythril_amd.engine import prepare
    from mythril_amd.smt2 import parse_script, to_smt2
    from tests.laser_concolic import run_sequence

    printed = {"s": 0.0}

    def sexpr(raws):                    # stands in for z3's Solver.sexpr(): not timed
        t = time.perf_counter()
        txt = to_smt2([r.node for r in raws])
        printed["s"] += time.perf_counter() - t
        return txt
    z3bridge.solver_sexpr = sexpr
    from tests import fakez3
    z = fakez3.module()
    sys.modules["z3"] = z
    rows = []
    for contract, scenarios in SCENARIOS.items():
        code = load_code(contract)
        for name, txs, *opt in scenarios:
            tag = f"{contract}/{name}"
            if a.only and a.only not in tag:
                continue
            opts = opt[0] if opt else {}
            _, run = run_sequence(code, txs, storage=opts.get("storage"), balances=scenario_balances(opts))
            cache = z3bridge.ConjunctCache(walk=not a.print)
            for qi, q in enumerate(run.queries):
                rs = [z.ast(n) for n in q.constraints]
                text = to_smt2(q.constraints)
                t0 = time.perf_counter()
                sw = parse_script(text)
                t1 = time.perf_counter()
                pw = prepare(sw.asserts, sw.ctx)
                t2 = time.perf_counter()
                printed["s"] = 0.0
                sc = cache.to_ir(rs)
                t3 = time.perf_counter()
                tm = {}
                pc = prepare(sc.asserts, sc.ctx, timings=tm)
                t4 = time.perf_counter()
                row = {"scenario": tag, "q": qi, "kind": q.kind, "conjuncts": len(rs),
                       "whole_parse": (t1 - t0) * 1e3, "whole_prepare": (t2 - t1) * 1e3,
                       "cached_parse": (t3 - t2 - printed["s"]) * 1e3, "cached_prepare": (t4 - t3) * 1e3}
                row.update({f"cached_{k}": v * 1e3 for k, v in tm.items()})
                row["whole"] = row["whole_parse"] + row["whole_prepare"]
                row["cached"] = row["cached_parse"] + row["cached_prepare"]
                if not a.no_check:
                    row["identical"] = program_bytes(pw.program) == program_bytes(pc.program)
                rows.append(row)
            print(f"{tag}: {len(run.queries)} queries, cache {cache.stats}", flush=True)
    keys = ("whole_parse", "whole_prepare", "whole", "cached_parse", "cached_prepare", "cached", "cached_lower",
            "cached_pools", "cached_compile")
    summary = {k: round(statistics.median(r[k] for r in rows), 4) for k in keys}
    summary["queries"] = len(rows)
    if not a.no_check:
        summary["identical"] = sum(r["identical"] for r in rows)
    print(json.dumps({"median_ms": summary}), flush=True)
    if a.out:
        json.dump({"rows": rows, "median_ms": summary}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
