#!/usr/bin/env python3
"""Where an assembled kernel and the asm interpreter disagree (GPU diagnostic).

    python tools/asmjit_diff.py FILE [FILE...] [--n 14] [--seed S]

For each corpus file: verdicts of both engines and the oracle over 2^n
generated candidates, the differing indices (count, blocks of 256, first
indices), which side matches the oracle, and the body's spill layout."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from mythril_amd import asmgen, asmjit  # noqa: E402
from mythril_amd.engine import DEFAULT_SEED, prepare  # noqa: E402
from mythril_amd.runtime import Device  # noqa: E402
from mythril_amd.smt2 import parse_file  # noqa: E402
from oracle import cdag  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--n", type=int, default=14)
    ap.add_argument("--seed", type=int, default=DEFAULT_SEED)
    a = ap.parse_args()
    dev = Device(0)
    n = 1 << a.n
    for f in a.files:
        s = parse_file(f)
        q = prepare(s.asserts, s.ctx)
        p = q.program
        di, da = dev.load(p), dev.load(p)
        asmjit.attach(dev, da, cache=False)
        va, _ = dev.eval_generated(da, a.seed, 0, n, trace=False)
        vi, _ = dev.eval_generated(di, a.seed, 0, n, trace=False)
        di.free()
        da.free()
        _, _, vo = cdag.evaluate(q.lowered.conjuncts, a.seed, 0, n, want_verdict=True,
                                 specs=cdag.program_specs(p))
        d = np.nonzero(va != vi)[0]
        print(os.path.basename(f), f"n_spill={p.n_spill} pool_words={len(p.pool)} "
              f"nlds={asmgen.lds_spill_words(p.n_spill, len(p.pool))}")
        print("  differ:", d.size, "blocks:", sorted(set((d // 256).tolist()))[:20], "first:", d[:16].tolist())
        print("  interp==oracle:", int(np.count_nonzero(vi.astype(np.uint8) == vo)), "of", n,
              " assembled==oracle:", int(np.count_nonzero(va.astype(np.uint8) == vo)))
        if d.size:
            print("  assembled verdicts there:", va[d[:16]].tolist(), "interp:", vi[d[:16]].tolist(),
                  "oracle:", vo[d[:16]].tolist())
    dev.close()


if __name__ == "__main__":
    main()
