"""One exhaustive interpreter launch of a solver-log query (PMC profiling aid).

    python tools/interp_once.py FILE [log2_candidates]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mythril_amd.engine import prepare  # noqa: E402
from mythril_amd.runtime import Device  # noqa: E402
from mythril_amd.smt2 import parse_file  # noqa: E402

s = parse_file(sys.argv[1])
q = prepare(s.asserts, s.ctx)
n = 1 << int(sys.argv[2] if len(sys.argv) > 2 else 22)
dev = Device(0)
dp = dev.load(q.program)
t0 = time.perf_counter()
found, st = dev.search([dp], 1, 0, n, 0)
print(os.path.basename(sys.argv[1]), "insns", q.program.n_insn, "cands", n, "kernel_ms", st["kernel_ms"],
      "wall_ms", (time.perf_counter() - t0) * 1e3, flush=True)
dp.free()
dev.close()
