#!/usr/bin/env python3
"""HBM traffic per launch of the benchmarked kernel from rocprofv3 PMC passes.

    python tools/pmc_traffic.py FETCH.csv WRITE.csv --kernel mwj_<sig> \
        --ops-per-eval N --batch B [--valu-csv SQ.csv] [--out profiles/pmc_traffic.json]

FETCH_SIZE and WRITE_SIZE come from separate `--pmc` passes (they do not fit
one pass: MI355X_MICROARCH.md counter table) and are in KiB.  On gfx950
FETCH_SIZE counts half of the bytes of a wide coalesced read, so

    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024

(cdna_hip_programming.md counter pitfalls; MI355X_MICROARCH.md §HBM), averaged
over the dispatches of the named kernel.  --valu-csv (a pass holding
SQ_INSTS_VALU and SQ_WAVES) adds the VALU wave-instructions per launch, from
which bench.py reports the VALU issue fraction (issued / 2.0 per CU-clock).
"""
import argparse
import csv
import json


def per_dispatch(path, counter, kernel):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter and row["Kernel_Name"].startswith(kernel):
                vals.append(float(row["Counter_Value"]))
    if not vals:
        raise SystemExit(f"{path}: no {counter} rows for kernel {kernel}")
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--ops-per-eval", type=int, required=True)
    ap.add_argument("--batch", type=int, required=True)
    ap.add_argument("--out", default=None)
    ap.add_argument("--note", default="")
    ap.add_argument("--valu-csv", default=None)
    ap.add_argument("--waves-csv", default=None)
    a = ap.parse_args()
    fetch = per_dispatch(a.fetch_csv, "FETCH_SIZE", a.kernel)
    write = per_dispatch(a.write_csv, "WRITE_SIZE", a.kernel)
    f_kib = sum(fetch) / len(fetch)
    w_kib = sum(write) / len(write)
    rec = {
        "kernel_name": a.kernel,
        "ops_per_eval": a.ops_per_eval,
        "batch": a.batch,
        "fetch_size_kib": f_kib,
        "write_size_kib": w_kib,
        "dispatches": [len(fetch), len(write)],
        "hbm_bytes_per_launch": int(round((2 * f_kib + w_kib) * 1024)),
        "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes; "
                  "(2*FETCH_SIZE + WRITE_SIZE) * 1024 bytes (KiB counters, gfx950 FETCH_SIZE counts half "
                  "of streamed reads: MI355X_MICROARCH.md §HBM)",
        "sources": [a.fetch_csv, a.write_csv],
    }
    if a.valu_csv:
        valu = per_dispatch(a.valu_csv, "SQ_INSTS_VALU", a.kernel)
        # SQ_WAVES: from the same pass, or from --waves-csv (gpu_run.sh pmc puts it in pass 1)
        waves = per_dispatch(a.waves_csv or a.valu_csv, "SQ_WAVES", a.kernel)
        rec["sq_insts_valu_per_launch"] = sum(valu) / len(valu)
        rec["sq_waves_per_launch"] = sum(waves) / len(waves)
        rec["sources"].append(a.valu_csv)
        if a.waves_csv:
            rec["sources"].append(a.waves_csv)
    if a.note:
        rec["note"] = a.note
    s = json.dumps(rec, indent=1)
    if a.out:
        open(a.out, "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
