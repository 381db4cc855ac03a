#!/usr/bin/env python3
"""Ground truth for the LASER corpus's "unknown" queries.

Every query of tests/golden/laser whose status is ``unknown`` (a not-followed
successor or a module query the concolic model does not satisfy) is searched
on the device in stages - 2^24 candidates, then 2^28, then 2^32 (launches of
2^30 from successive offsets) - with stop-after-hit, and every witness found
is checked against the ORIGINAL formula by the oracle (oracle/dag_eval).  The
witnesses are written to a JSON file (tests/golden/laser/ground_truth.json
once committed), so the CPU suite re-checks them without a GPU
(tests/test_laser_corpus.py::test_ground_truth_witnesses_hold).

    python tools/ground_truth.py --out gpurun_out/gt/ground_truth.json [--max-log2 32]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mythril_amd.engine import WitnessEngine, prepare  # noqa: E402
from mythril_amd.smt2 import parse_file  # noqa: E402
from tests.test_engine_cpu import holds  # noqa: E402

CORPUS = os.path.join(ROOT, "tests", "golden", "laser")


def witness_json(w) -> dict:
    return {"index": w.index,
            "values": {k: hex(v) for k, v in sorted(w.values.items())},
            "arrays": {k: {hex(i): hex(v) for i, v in sorted(c.items())} for k, c in sorted(w.arrays.items())},
            "functions": {k: [[[hex(a) for a in args], hex(v)] for args, v in sorted(t.items())]
                          for k, t in sorted(w.functions.items())}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--max-log2", type=int, default=32)
    ap.add_argument("--only", default=None, help="substring of the file names to search")
    a = ap.parse_args()
    man = json.load(open(os.path.join(CORPUS, "manifest.json")))
    todo = [m for m in man if m["status"] == "unknown" and (a.only is None or a.only in m["file"])]
    print(f"{len(todo)} unknown queries", flush=True)
    eng = WitnessEngine(device=0, budget=1 << 24, op_budget=None)
    out = {"stages": [], "witnessed": {}, "no_witness": []}
    qs = []
    for m in todo:
        s = parse_file(os.path.join(CORPUS, m["file"]))
        qs.append((m, s, prepare(s.asserts, s.ctx)))
    left = qs
    stages = [(24, 64, 24), (28, 16, 28)] + [(30, 4, a.max_log2)] if a.max_log2 > 28 else [(24, 64, 24), (28, 16, 28)]
    for log2, per_launch, upto in stages:
        t0 = time.perf_counter()
        nxt = []
        for i in range(0, len(left), per_launch):
            chunk = left[i:i + per_launch]
            found = [None] * len(chunk)
            begin = 0
            while begin < (1 << upto):
                open_ix = [j for j, w in enumerate(found) if w is None]
                if not open_ix:
                    break
                ws = eng.search([chunk[j][2] for j in open_ix], count=1 << log2, begin=begin)
                for j, w in zip(open_ix, ws):
                    found[j] = w
                begin += 1 << log2
                print(f"  stage 2^{upto}: queries {i}-{i + len(chunk)} offset 2^{begin.bit_length() - 1} "
                      f"({time.perf_counter() - t0:.1f} s)", flush=True)
            for (m, s, q), w in zip(chunk, found):
                if w is None:
                    nxt.append((m, s, q))
                    continue
                assert holds(s.asserts, w), m["file"]      # the oracle, on the original formula
                d = witness_json(w)
                d["searched_log2"] = upto
                out["witnessed"][m["file"]] = d
        out["stages"].append({"log2": upto, "searched": len(left), "witnessed": len(left) - len(nxt),
                              "seconds": round(time.perf_counter() - t0, 2)})
        print(f"stage 2^{upto}: {len(left) - len(nxt)} of {len(left)} witnessed", flush=True)
        left = nxt
        if not left:
            break
    out["no_witness"] = [m["file"] for m, _, _ in left]
    out["kernel_ms"] = round(eng.stats["kernel_ms"], 1)
    eng.close()
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    json.dump(out, open(a.out, "w"), indent=1, sort_keys=True)
    print(f"{len(out['witnessed'])} witnessed, {len(left)} without a witness at 2^{a.max_log2}", flush=True)


if __name__ == "__main__":
    main()
