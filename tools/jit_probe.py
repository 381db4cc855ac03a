#!/usr/bin/env python3
"""Diagnostic: localise a specialised-kernel vs interpreter disagreement inside
one conjunct of bench.py's C5 program.  For every division node (and a sample
of the other nodes) of conjunct C, a probe program asserts `node == value`,
with the value the host build computes at candidate I; the specialised kernel
and the interpreter evaluate every probe over the 64-candidate wave holding I.
The first probe whose kernel verdict at I differs names the node.

Usage: python tools/jit_probe.py C I [--compile-only]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mythril_amd import hostemu, jit  # noqa: E402
from mythril_amd.compiler import compile_program  # noqa: E402
from mythril_amd.ir import BOOL, topo  # noqa: E402
from mythril_amd.synth import build_c5  # noqa: E402


def main():
    ci, idx = int(sys.argv[1]), int(sys.argv[2])
    syn = build_c5(hostemu.term_values)
    conj = syn.conjuncts[ci]
    nodes = [n for n in topo([conj]) if n.op not in ("var", "const")]
    pick = [n for n in nodes if n.op in ("bvudiv", "bvurem")]
    pick += nodes[:: max(1, len(nodes) // 12)] + [nodes[-1]]
    pick = sorted(set(pick), key=nodes.index)
    vals = hostemu.term_values(pick, idx, syn.seed)
    c = syn.ctx
    progs = []
    for n, v in zip(pick, vals):
        if n.width == BOOL or getattr(n, "sort", None) == BOOL:
            t = n if v else c.app("not", n)
        else:
            t = c.app("=", n, c.const(v, n.width))
        progs.append(compile_program([t]))
    image, names, dt = jit.compile_device(progs, "x", waves=2, lds_leaves=10)
    print(f"{len(progs)} probes compiled in {dt:.0f} s", flush=True)
    if "--compile-only" in sys.argv:
        return
    from mythril_amd.runtime import Device
    dev = Device(0)
    begin = idx - (idx - (syn.witness_index - 32768)) % 64   # the wave holding idx in jit_check's window
    for n, p, name in zip(pick, progs, names):
        s = dev.load(p)
        dev.attach_kernel(s, image, name)
        i = dev.load(p)
        vs, _ = dev.eval_generated(s, syn.seed, begin, 64, trace=False)
        vi, _ = dev.eval_generated(i, syn.seed, begin, 64, trace=False)
        k = idx - begin
        print(f"node {n.id:6d} {n.op:10s} pos {nodes.index(n):4d}: interpreter {int(vi[k])} specialised {int(vs[k])}"
              f"{'   <-- differs' if vi[k] != vs[k] else ''}", flush=True)
        s.free()
        i.free()


if __name__ == "__main__":
    main()
