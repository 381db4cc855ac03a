#!/usr/bin/env python3
"""Diagnostic: the C5 bench program's verdict at its planted witness index on
the host build (hostemu, which planted it), the device interpreter and the
specialised kernel; per conjunct when they disagree."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mythril_amd import hostemu, jit  # noqa: E402
from mythril_amd.compiler import compile_program  # noqa: E402
from mythril_amd.runtime import Device  # noqa: E402
from mythril_amd.synth import build_c5  # noqa: E402


def main():
    syn = build_c5(hostemu.term_values)
    if "--compile-only" in sys.argv:
        jit.compile_parts(compile_program(syn.conjuncts), "x", waves=2, lds_leaves=jit.BENCH_LDS_LEAVES)
        return
    w = syn.witness_index
    p = compile_program(syn.conjuncts)
    dev = Device(0)
    interp = dev.load(p)
    special = dev.load(p)
    jit.attach(dev, [special], variants="x", waves=2, lds_leaves=jit.BENCH_LDS_LEAVES)
    split = dev.load(p)
    jit.attach(dev, [split], variants="x", waves=2, lds_leaves=jit.BENCH_LDS_LEAVES, split=True)
    vi, _ = dev.eval_generated(interp, syn.seed, w, 1, trace=False)
    vs, _ = dev.eval_generated(special, syn.seed, w, 1, trace=False)
    vp, _ = dev.eval_generated(split, syn.seed, w, 1, trace=False)
    print(f"split kernels ({split.kernel}): {int(vp[0])}", flush=True)
    import numpy as np
    n = 1 << 17
    ai, _ = dev.eval_generated(interp, syn.seed, w - n // 2, n, trace=False)
    aS, _ = dev.eval_generated(special, syn.seed, w - n // 2, n, trace=False)
    aP, _ = dev.eval_generated(split, syn.seed, w - n // 2, n, trace=False)
    print(f"window of {n}: interpreter {int(ai.sum())} satisfied, specialised {int(aS.sum())}, split {int(aP.sum())}; "
          f"mismatches specialised {int(np.count_nonzero(ai != aS))}, split {int(np.count_nonzero(ai != aP))}",
          flush=True)
    host = hostemu.term_values(syn.conjuncts, w, syn.seed)
    print(f"planted {w}: host {[int(h) for h in host].count(1)}/{len(host)} conjuncts true, "
          f"interpreter {int(vi[0])}, specialised {int(vs[0])}", flush=True)
    # chain ends and every division result at the witness: host vs device interpreter trace
    from mythril_amd.ir import topo
    divs = [n for n in topo(syn.chain_ends) if n.op in ("bvudiv", "bvurem")]
    hv = hostemu.term_values(divs, w, syn.seed)
    tp = compile_program([], trace=divs)
    dp = dev.load(tp)
    from mythril_amd.runtime import unpack_trace
    _, tr = dev.eval_generated(dp, syn.seed, w, 1)
    bad = 0
    for n, h in zip(divs, hv):
        d = unpack_trace(tp, tr, n)[0]
        if d != h:
            bad += 1
            if bad <= 5:
                print(f"  {n.op} node {n.id}: host {h:#x} device {d:#x}", flush=True)
    print(f"division results differing host vs device interpreter: {bad} of {len(divs)}", flush=True)


if __name__ == "__main__":
    main()
