#!/usr/bin/env python3
"""Diagnostic: asm interpreter vs compiled interpreter verdicts on every query
of the concolic corpus runs (tests/laser_replay.py), programs built the way
the drop-in builds them (prepare on the recorded constraint lists)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mythril_amd import isa  # noqa: E402
from mythril_amd.engine import DEFAULT_SEED, prepare  # noqa: E402
from mythril_amd.runtime import Device  # noqa: E402
from tests.laser_replay import concolic_runs  # noqa: E402

dev = Device(0)
n = 1 << 14
bad = 0
inv = {v: k for k, v in isa.OPCODES.items()}
for name, m, run, ntx in concolic_runs():
    for qi, q in enumerate(run.queries):
        p = prepare(q.constraints, m.c).program
        dp = dev.load(p)
        os.environ["MYTHRIL_AMD_ASM"] = "1"
        eng = dev.engine_of(dp)
        va, _ = dev.eval_generated(dp, DEFAULT_SEED, 0, n, trace=False)
        os.environ["MYTHRIL_AMD_ASM"] = "0"
        vi, _ = dev.eval_generated(dp, DEFAULT_SEED, 0, n, trace=False)
        dp.free()
        d = np.nonzero(va != vi)[0]
        if d.size:
            bad += 1
            ops = sorted({inv[int(w) & 0xff] for w in list(p.code)[0::4]})
            print(f"{name} q{qi}: {d.size} mismatches, first {d[:8].tolist()} asm={va[d[:8]].tolist()} "
                  f"interp={vi[d[:8]].tolist()} engine={eng} insns={p.n_insn} spill={p.n_spill} "
                  f"npool={p.pool.size} ops={ops}", flush=True)
print("programs with mismatches:", bad, flush=True)

# searches as the drop-in issues them: JUMPI pairs in one launch, early exit +
# stop after hit, the default budget; every reported index re-evaluated
from mythril_amd.engine import DEFAULT_BUDGET  # noqa: E402
flags = isa.FLAG_EARLY_EXIT | isa.FLAG_STOP_AFTER_HIT
sbad = 0
for name, m, run, ntx in concolic_runs():
    qs = run.queries
    i = 0
    while i < len(qs):
        grp = [qs[i]]
        if i + 1 < len(qs) and qs[i + 1].pc == qs[i].pc and qs[i + 1].tx == qs[i].tx:
            grp.append(qs[i + 1])
        progs = [prepare(q.constraints, m.c).program for q in grp]
        dps = [dev.load(p) for p in progs]
        res = {}
        for eng in ("1", "0"):
            os.environ["MYTHRIL_AMD_ASM"] = eng
            res[eng], _ = dev.search(dps, DEFAULT_SEED, 0, DEFAULT_BUDGET, flags)
        for k, (dp, fa, fi) in enumerate(zip(dps, res["1"], res["0"])):
            checks = []
            for f in (fa, fi):
                if f is not None:
                    os.environ["MYTHRIL_AMD_ASM"] = "0"
                    v, _ = dev.eval_generated(dp, DEFAULT_SEED, f, 1, trace=False)
                    checks.append(int(v[0]))
            if fa != fi or 0 in checks:
                sbad += 1
                print(f"SEARCH {name} q{i + k}: asm {fa} interp {fi} re-eval {checks} group {len(grp)}", flush=True)
        for dp in dps:
            dp.free()
        i += len(grp)
print("search mismatches:", sbad, flush=True)
