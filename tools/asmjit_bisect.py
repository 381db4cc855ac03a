#!/usr/bin/env python3
"""Find the conjunct where an assembled kernel first disagrees with the asm
interpreter (GPU diagnostic): prefixes of the lowered conjunction, compiled
with the full program's leaf layout (same candidates), bisected on the
indices where the full programs differ.

    python tools/asmjit_bisect.py FILE [--n 14]"""
import argparse
import dataclasses
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from mythril_amd import asmgen, asmjit, isa  # noqa: E402
from mythril_amd.compiler import compile_program  # noqa: E402
from mythril_amd.engine import DEFAULT_SEED, prepare  # noqa: E402
from mythril_amd.runtime import Device  # noqa: E402
from mythril_amd.smt2 import parse_file, to_smt2  # noqa: E402


def verdicts(dev, p, n, seed):
    di, da = dev.load(p), dev.load(p)
    try:
        asmjit.attach(dev, da, cache=False)
        va, _ = dev.eval_generated(da, seed, 0, n, trace=False)
        vi, _ = dev.eval_generated(di, seed, 0, n, trace=False)
    finally:
        di.free()
        da.free()
    return va, vi


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("file")
    ap.add_argument("--n", type=int, default=14)
    ap.add_argument("--tail", type=int, default=0, help="print the last TAIL instructions of the first "
                    "differing prefix and their assembled body")
    a = ap.parse_args()
    n, seed = 1 << a.n, DEFAULT_SEED
    s = parse_file(a.file)
    q = prepare(s.asserts, s.ctx)
    conj = q.lowered.conjuncts
    fixed = {sp.name: dataclasses.replace(sp, pool=None if sp.pool is None else list(sp.pool))
             for sp in q.program.leaf_specs}
    dev = Device(0)
    va, vi = verdicts(dev, q.program, n, seed)
    bad = np.nonzero(va != vi)[0]
    print("full program: differ", bad.size, "conjuncts", len(conj), flush=True)
    if not bad.size:
        return

    def differs(k):
        p = compile_program(conj[:k], leaf_specs=fixed)
        x, y = verdicts(dev, p, n, seed)
        return bool(np.any(x != y))

    lo, hi = 0, len(conj)        # differs(hi) holds, differs(lo) does not
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if differs(mid):
            hi = mid
        else:
            lo = mid
        print("  prefix", mid, "differs" if hi == mid else "agrees", flush=True)
    c = conj[hi - 1]
    print("first differing conjunct:", hi - 1)
    print(to_smt2([c])[-3000:])
    p1 = compile_program([c], leaf_specs=fixed)
    x, y = verdicts(dev, p1, n, seed)
    print("alone: differ", int(np.count_nonzero(x != y)))
    names = {v: k for k, v in isa.OPCODES.items()}
    if a.tail:
        p1 = compile_program(conj[:hi], leaf_specs=fixed)   # in context: the tail of the first differing prefix
        print(f"prefix {hi}: {len(p1.code) // 4} instructions, n_spill {p1.n_spill}, pool {len(p1.pool)}")
    ni = len(p1.code) // 4
    first = max(0, ni - a.tail) if a.tail else 0
    for i in range(first, ni):
        w = [int(t) for t in p1.code[4 * i:4 * i + 4]]
        print(f"  {i:4d} {names[w[0] & 0xff]:12s} w={w[0] >> 16:3d} dst={w[1] & 0xffff:#06x} "
              f"a={w[1] >> 16:#06x} b={w[2] & 0xffff:#06x} c={w[2] >> 16:#06x} imm={w[3]:#x}")
    body = asmgen.static_body(p1.code, p1.consts, p1.leaves, nlds=asmgen.lds_spill_words(p1.n_spill, len(p1.pool)),
                              pool=p1.pool)
    start = next((j for j, ln in enumerate(body) if ln.startswith(f"; {first}:")), 0)
    print("\n".join(body[start:start + 1500]))
    dev.close()


if __name__ == "__main__":
    main()
