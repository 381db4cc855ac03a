#!/usr/bin/env python3
"""Per-bytecode-instruction counters from tools/interp_opcost.py's PMC pass,
for each interpreter kernel (mw_search_asm_kernel: the threaded-dispatch asm
interpreter; mw_search_kernel: the compiled one).  Every variant runs a warm-up
and a measured launch per engine; the measured one is used.

    python tools/opcost_summary.py TAG      (reads gpurun_out/TAG/opcost_pmc)
"""
import collections
import csv
import glob
import sys

NAMES = ["CHECK", "CHECK_IMPEQ_regs", "CHECK_IMPEQ_const", "N_ADD", "N_EQN", "MOV_N", "N_EQ_wide", "W_ADD", "W_AND",
         "LEAF_N", "LEAF_W"]


def main():
    tag = sys.argv[1]
    log2 = int(sys.argv[2]) if len(sys.argv) > 2 else 18
    path = glob.glob(f"gpurun_out/{tag}/opcost_pmc/**/*counter_collection.csv", recursive=True)[0]
    rows = collections.defaultdict(dict)
    kern = {}
    for row in csv.DictReader(open(path)):
        if "mw_search" in row["Kernel_Name"]:
            d = int(row["Dispatch_Id"])
            rows[d][row["Counter_Name"]] = float(row["Counter_Value"])
            kern[d] = "asm" if "asm" in row["Kernel_Name"] else "interp"
    for engine in ("asm", "interp"):
        ids = sorted(d for d in rows if kern[d] == engine)
        for k, name in enumerate(NAMES):
            if 2 * k + 1 >= len(ids):
                break
            r = rows[ids[2 * k + 1]]
            rep = 500 if name.startswith("LEAF") else 2000
            w = r["SQ_WAVES"]
            chunks = (1 << log2) // 64 / w

            def per(c):
                return r[c] / w / chunks / rep
            print(f"{engine:6s} {name:18s} VALU {per('SQ_INSTS_VALU'):6.1f} SALU {per('SQ_INSTS_SALU'):6.1f} "
                  f"SMEM {per('SQ_INSTS_SMEM'):5.2f} BR {per('SQ_INSTS_BRANCH'):5.1f} cyc {per('SQ_WAVE_CYCLES'):7.1f}")


if __name__ == "__main__":
    main()
