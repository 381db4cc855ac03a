#!/usr/bin/env python3
"""Experiment helper: compile bench.py's C5 kernel with non-default code
generation options into build/jit (MW_JIT_SPLIT=branch|sched_barrier env,
--interleave K, --waves W, --lds L), for an A/B run of bench.py on the GPU."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

ap = argparse.ArgumentParser()
ap.add_argument("--interleave", type=int, default=1)
ap.add_argument("--waves", type=int, default=2)
ap.add_argument("--lds", type=int, default=10)
ap.add_argument("--nodes", type=int, default=10000)
a = ap.parse_args()
from mythril_amd import hostemu, jit  # noqa: E402
from mythril_amd.compiler import compile_program  # noqa: E402
from mythril_amd.synth import build_c5  # noqa: E402
syn = build_c5(hostemu.term_values, n_nodes=a.nodes)
p = compile_program(syn.conjuncts)
t = time.time()
_, names, dt = jit.compile_device([p], "x", waves=a.waves, lds_leaves=a.lds, interleave=a.interleave)
print(f"{names[0]} split={jit.SPLIT_KIND} interleave={a.interleave} waves={a.waves} lds={a.lds}: "
      f"{'compiled in %.0f s' % dt if dt else 'cached'}", flush=True)
