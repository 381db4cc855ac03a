#!/usr/bin/env python3
"""Run one interpreter microbenchmark (op chain, no spills) a few times for PMC passes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from opbench import chain  # noqa: E402
from mythril_amd.compiler import compile_program  # noqa: E402
from mythril_amd.runtime import Device  # noqa: E402

op = sys.argv[1] if len(sys.argv) > 1 else "bvxor"
dev = Device(0)
c, conj = chain(op, n=400)
p = compile_program(conj)
dp = dev.load(p)
for _ in range(3):
    (_,), st = dev.search([dp], 1, 0, 1 << 20, 0)
print(op, p.n_insn, st["kernel_ms"])
