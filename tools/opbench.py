#!/usr/bin/env python3
"""Per-op-class throughput of the interpreter or the specialised kernels (diagnostic).

Usage: python tools/opbench.py [interp|jit]

For each op class, a program of one long dependent chain over 4 leaves (no
spills) is searched exhaustively; reports evals/s, algorithmic Tops/s and the
fraction of the measured VALU peak, plus the measured peaks themselves.
Writes gpurun_out/opbench.json.
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mythril_amd.compiler import compile_program  # noqa: E402
from mythril_amd.ir import Ctx  # noqa: E402
from mythril_amd.runtime import Device  # noqa: E402


OPS = ["bvadd", "bvsub", "bvxor", "bvand", "bvmul", "bvult", "=", "ite", "bvshl", "bvlshr", "bvashr",
       "extract", "bvudiv", "bvurem"]


def chain(op, w=256, n=400, nleaves=4):
    c = Ctx()
    xs = [c.var(f"x{i}", w) for i in range(nleaves)]
    prev = xs[0]
    for i in range(n):
        o = xs[(i + 1) % nleaves]
        if op == "ite":
            prev = c.app("ite", c.app("bvult", prev, o), prev, o)
        elif op in ("bvult", "="):
            prev = c.app("ite", c.app(op, prev, o), o, prev)
        elif op in ("bvudiv", "bvurem"):
            prev = c.app(op, prev, c.app("bvor", o, c.const(1, w)))
        elif op in ("bvshl", "bvlshr", "bvashr"):
            prev = c.app(op, prev, c.app("bvand", o, c.const(255, w)))
        elif op == "extract":
            prev = c.app("concat", c.app("extract", prev, params=(w // 2 + 63, 64)),
                         c.app("extract", o, params=(w // 2 - 1, 0)))
        else:
            prev = c.app(op, prev, o)
    return c, [c.app("bvult", prev, c.const(5, w))]


def main():
    engine = sys.argv[1] if len(sys.argv) > 1 else "interp"
    dev = Device(0)
    res = {"engine": engine}
    for mul in (False, True):
        ops, ms = dev.valu_peak(mul)
        res["peak_mul" if mul else "peak_add"] = {"ops_per_s": ops, "kernel_ms": ms}
        print(f"peak {'v_mul_lo_u32' if mul else 'v_add_u32'}: {ops/1e12:.2f} T/s ({ms:.2f} ms)", flush=True)
    peak = res["peak_add"]["ops_per_s"]
    count = 1 << 20
    for op in OPS:
        n = 50 if op in ("bvudiv", "bvurem") else 400
        c, conj = chain(op, n=n)
        p = compile_program(conj)
        dp = dev.load(p)
        if engine == "jit":
            from mythril_amd import jit
            # chain values pass through an opaque copy: no folding across nodes
            image, names, _ = jit.compile_device([p], "x", fence_first=True)
            dev.attach_kernel(dp, image, names[0])
        dev.search([dp], 1, 0, count, 0)
        (_,), st = dev.search([dp], 1, 0, count, 0)
        evs = count / (st["kernel_ms"] / 1e3)
        ach = evs * p.ops_per_eval
        res[op] = {"insns": p.n_insn, "ops_per_eval": p.ops_per_eval, "kernel_ms": st["kernel_ms"],
                   "evals_per_s": evs, "Tops": ach / 1e12, "frac_peak": ach / peak,
                   "insn_per_s_per_lane": evs * p.n_insn}
        print(f"{op:8s} insns={p.n_insn:5d} ops/eval={p.ops_per_eval:7d} {st['kernel_ms']:8.2f} ms "
              f"{evs/1e6:8.2f} Mevals/s {ach/1e12:6.2f} Tops/s {100*ach/peak:5.1f}% "
              f"insn-rate {evs*p.n_insn/1e9:6.1f} G/s", flush=True)
        dp.free()
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open(f"gpurun_out/opbench_{engine}.json", "w"), indent=1)


if __name__ == "__main__":
    main()
