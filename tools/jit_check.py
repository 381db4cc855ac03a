#!/usr/bin/env python3
"""Diagnostic: specialised kernel vs interpreter verdicts on a small C5-shaped
program (mixed verdicts), per conjunct.  Compile on the CPU with --compile-only,
then run on the GPU box.  Prints the mismatch count of the whole program and
of each conjunct program (the first mismatching conjunct localises an ALU bug).

Usage: python tools/jit_check.py [--nodes N] [--conj K] [--compile-only]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from mythril_amd import hostemu, jit  # noqa: E402
from mythril_amd.compiler import compile_program  # noqa: E402
from mythril_amd.synth import build_c5  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=640)
    ap.add_argument("--conj", type=int, default=8)
    ap.add_argument("--count", type=int, default=1 << 16)
    ap.add_argument("--compile-only", action="store_true")
    ap.add_argument("--no-full", action="store_true", help="conjunct programs only (no whole-program kernel)")
    ap.add_argument("--flags", default="", help="extra device flags for the specialised kernels (experiments)")
    ap.add_argument("--bench", action="store_true",
                    help="bench.py's C5 program (density 2^-24, leftover comparisons kept), checked around the witness")
    a = ap.parse_args()
    jit.EXTRA_FLAGS = a.flags.split()
    if a.bench:
        syn = build_c5(hostemu.term_values, n_nodes=a.nodes, n_conj=a.conj)
    else:
        syn = build_c5(hostemu.term_values, n_nodes=a.nodes, n_conj=a.conj, density_log2=1, keep_pending=False)
    begin = syn.witness_index - a.count // 2 if a.bench else 0
    progs = [compile_program(syn.conjuncts)] + [compile_program([c]) for c in syn.conjuncts]
    if a.no_full:
        progs = progs[1:]
    image, names, dt = jit.compile_device(progs, "x", waves=2, lds_leaves=10)
    print(f"compiled {len(progs)} programs in {dt:.0f} s", flush=True)
    if a.compile_only:
        return
    from mythril_amd.runtime import Device
    dev = Device(0)
    bad = 0
    for k, (p, name) in enumerate(zip(progs, names)):
        s = dev.load(p)
        dev.attach_kernel(s, image, name)
        i = dev.load(p)
        vs, _ = dev.eval_generated(s, syn.seed, begin, a.count, trace=False)
        vi, _ = dev.eval_generated(i, syn.seed, begin, a.count, trace=False)
        mism = int(np.count_nonzero(vs != vi))
        if mism and a.bench:
            extra_idx = (np.nonzero(vs != vi)[0][:4] + begin).tolist()
            print(f"  first mismatching indices {extra_idx} (witness {syn.witness_index})", flush=True)
        bad += mism
        extra = ""
        print(f"{'program' if k == 0 and not a.no_full else 'conjunct %d' % (k - (0 if a.no_full else 1))}: {mism} mismatches of {a.count}, "
              f"{int(vi.sum())} satisfied (interpreter){extra}", flush=True)
        s.free()
        i.free()
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
