#!/usr/bin/env python3
"""Where an interpreter program's time goes: run a query's program with
classes of instructions removed (results are meaningless; only the kernel
time is read) and print the kernel time of each variant.

    python tools/c3_ablate.py [FILE] [--log2 22]
"""
import argparse
import copy
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mythril_amd import isa  # noqa: E402

INV = {v: k for k, v in isa.OPCODES.items()}


def without(p, drop):
    code = p.code.reshape(-1, 4)
    keep = [r for r in code if INV[int(r[0]) & 0xFF] not in drop]
    q = copy.copy(p)
    q.code = np.ascontiguousarray(np.asarray(keep, dtype=np.uint32).reshape(-1))
    q.n_insn = len(keep)
    return q


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("file", nargs="?", default=os.path.join(ROOT, "tests", "golden", "solver_log",
                                                           "c3_bec_batchtransfer_overflow.smt2"))
    ap.add_argument("--log2", type=int, default=22)
    a = ap.parse_args()
    from mythril_amd.engine import prepare
    from mythril_amd.runtime import Device
    from mythril_amd.smt2 import parse_file
    s = parse_file(a.file)
    p = prepare(s.asserts, s.ctx).program
    ops = sorted({INV[int(r[0]) & 0xFF] for r in p.code.reshape(-1, 4)})
    checks = {"CHECK", "CHECK_IMP", "CHECK_IMPEQ", "CHECK_IMPEQW", "CHECK_IMPEQK"}
    spills = {"SPILL_W", "SPILL_N", "FILL_W", "FILL_N"}
    leaves = {"LEAF_W", "LEAF_N", "W_CDINS"}
    variants = {
        "full": set(),
        "no_impeq": {"CHECK_IMPEQ", "CHECK_IMPEQK"},
        "no_grid_rows": {"CHECK_GRID"},
        "no_leaf_n": {"LEAF_N"},
        "no_byte_inserts": {"N_SLT", "N_ITE", "W_INSN"},
        "no_checks": checks,
        "no_spills": spills,
        "no_checks_spills": checks | spills,
        "leaves_only": set(ops) - leaves - {"END"},
        "empty": set(ops) - {"END"},
    }
    dev = Device(0)
    n = 1 << a.log2
    for name, drop in variants.items():
        q = without(p, drop)
        dp = dev.load(q)
        dev.search([dp], 1, 0, n, 0)
        _, st = dev.search([dp], 1, 0, n, 0)
        dp.free()
        print(json.dumps({"variant": name, "insns": q.n_insn, "kernel_ms": round(st["kernel_ms"], 3),
                          "Mevals_s": round(n / st["kernel_ms"] / 1e3, 1)}), flush=True)
    dev.close()


if __name__ == "__main__":
    main()
