"""One exhaustive launch of a solver-log query (PMC profiling aid), on the
asm interpreter, (--jit) the query's cached specialised kernel, (--asmjit)
its assembled kernel or (--interp) the compiled interpreter.

    python tools/interp_once.py FILE [log2_candidates] [--jit | --asmjit | --interp]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mythril_amd.engine import prepare  # noqa: E402
from mythril_amd.runtime import Device  # noqa: E402
from mythril_amd.smt2 import parse_file  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
s = parse_file(args[0])
q = prepare(s.asserts, s.ctx)
n = 1 << int(args[1] if len(args) > 1 else 22)
dev = Device(0)
dp = dev.load(q.program)
if "--jit" in sys.argv:
    from mythril_amd import jit
    jit.attach(dev, [dp], variants="xe", waves=2, lds_leaves=0)
if "--asmjit" in sys.argv:
    from mythril_amd import asmjit
    asmjit.attach(dev, dp)
if "--interp" in sys.argv:
    os.environ["MYTHRIL_AMD_ASM"] = "0"
t0 = time.perf_counter()
found, st = dev.search([dp], 1, 0, n, 0)
print(os.path.basename(args[0]), "insns", q.program.n_insn, "cands", n, "engine", dev.engine_of(dp), "kernel_ms",
      st["kernel_ms"], "wall_ms", (time.perf_counter() - t0) * 1e3, flush=True)
dp.free()
dev.close()
