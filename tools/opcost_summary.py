#!/usr/bin/env python3
"""Per-bytecode-instruction counters from tools/interp_opcost.py's PMC pass
(gpurun_out/TAG/opcost_pmc, run with its log in gpurun_out/TAG/opcost_pmc.log):
every JSON line of the log is one (variant, engine) and owns two consecutive
search dispatches (warm-up, measured); the measured one is used.

    python tools/opcost_summary.py TAG
"""
import collections
import csv
import glob
import json
import sys


def main():
    tag = sys.argv[1]
    lines = [json.loads(ln) for ln in open(f"gpurun_out/{tag}/opcost_pmc.log") if ln.startswith("{")]
    path = glob.glob(f"gpurun_out/{tag}/opcost_pmc/**/*counter_collection.csv", recursive=True)[0]
    rows = collections.defaultdict(dict)
    for row in csv.DictReader(open(path)):
        if "mw_search" in row["Kernel_Name"]:
            rows[int(row["Dispatch_Id"])][row["Counter_Name"]] = float(row["Counter_Value"])
    # the context's introspection launches (one block per asm kernel) come first
    ids = [i for i in sorted(rows) if rows[i].get("SQ_WAVES", 0) > 16]
    for k, ln in enumerate(lines):
        if 2 * k + 1 >= len(ids):
            break
        r = rows[ids[2 * k + 1]]
        w = r["SQ_WAVES"]
        chunks = (1 << ln["log2"]) // 64 / w

        def per(c):
            return r[c] / w / chunks / ln["repeat"]
        print(f"{ln['engine']:6s} {ln['op']:22s} VALU {per('SQ_INSTS_VALU'):6.1f} SALU {per('SQ_INSTS_SALU'):6.1f} "
              f"SMEM {per('SQ_INSTS_SMEM'):5.2f} BR {per('SQ_INSTS_BRANCH'):5.1f} cyc {per('SQ_WAVE_CYCLES'):7.1f} "
              f"wait_inst {per('SQ_WAIT_INST_ANY'):6.1f} wait_any {per('SQ_WAIT_ANY'):6.1f}")


if __name__ == "__main__":
    main()
