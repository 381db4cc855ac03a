#!/usr/bin/env python3
"""Interpreter cost per bytecode instruction, by opcode (device microbenchmark).

Each variant is a hand-assembled program: a few leaves, then REPEAT copies of
one instruction, then END, searched exhaustively (flags 0) over 2^20
candidates.  Prints ns per instruction per wave-slot and, under rocprofv3
--pmc, the per-dispatch counters give VALU/SALU/SMEM instructions per
bytecode instruction.

    python tools/interp_opcost.py [--repeat 2000] [--log2 20] [--engines asm,interp]
"""
import argparse
import copy
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mythril_amd import isa  # noqa: E402
from mythril_amd.compiler import compile_program  # noqa: E402
from mythril_amd.ir import Ctx  # noqa: E402

K = isa.KBIT


def base_program(pooled=False):
    """4 narrow leaves (8-bit) and 2 wide ones, a narrow and two wide constants.
    pooled: the leaves draw from 8-entry pools (bit-interleaved digits, as
    the calldata bytes of Mythril's queries) instead of Philox."""
    c = Ctx()
    n = [c.var(f"n{i}", 8) for i in range(4)]
    w = [c.var(f"w{i}", 256) for i in range(2)]
    conj = [c.app("=", n[0], c.const(5, 8)), c.app("=", n[1], n[2]), c.app("=", n[3], n[0]),
            c.app("bvult", w[0], c.const(1 << 200, 256)), c.app("=", w[1], w[0]),
            c.app("bvult", w[1], c.const(0x24, 256))]
    pools = None
    if pooled:
        pools = {f"n{i}": [1, 2, 3, 5, 7, 11, 13, None] for i in range(4)}
        pools.update({f"w{i}": [0x44, 4, 1 << 255, None] for i in range(2)})
    return compile_program(conj, pools=pools)


def assemble(p, body, repeat):
    """Leaves into N0..N3 / W0..W1, then `body` (list of encoded insns) repeated."""
    idx = {n.name: i for i, n in enumerate(p.leaf_nodes)}
    code = []
    for i in range(4):
        code += isa.encode("LEAF_N", 8, isa.encode_dst("N", i), imm=idx[f"n{i}"])
    for i in range(2):
        code += isa.encode("LEAF_W", 256, isa.encode_dst("W", i), imm=idx[f"w{i}"])
    for _ in range(repeat):
        for ins in body:
            code += ins
    code += isa.encode("END", 0, isa.encode_dst(None))
    q = copy.copy(p)
    q.code = np.asarray(code, dtype=np.uint32)
    q.n_insn = len(code) // 4
    q.n_spill = 0
    q.stats = dict(p.stats)
    return q


def kn(p):
    """Constant-pool offset of a narrow constant (the program's 8-bit 5)."""
    return K | int(np.nonzero(p.consts == 5)[0][0])


def kw(p, val):
    """Constant-pool offset of the 256-bit constant val."""
    k = p.consts.reshape(-1)
    for o in range(0, len(k) - 7):
        if int(k[o]) == val and not k[o + 1:o + 8].any():
            return K | o
    raise KeyError(val)


def variants(p):
    def e(op, width=0, dst=0, a=0, b=0, c=0, imm=0):   # dst: a slot of the op's result file
        return isa.encode(op, width, isa.encode_dst(isa.SHAPES[op][0], dst), a, b, c, imm)
    idx = {n.name: i for i, n in enumerate(p.leaf_nodes)}
    return {
        "CHECK": [e("CHECK", 1, 0, 4)],
        "CHECK_IMPEQ_regs": [e("CHECK_IMPEQ", 8, 0, 4, 1, 2)],
        "CHECK_IMPEQ_const": [e("CHECK_IMPEQ", 8, 0, 4, 1, kn(p))],
        "CHECK_IMPEQK_regs": [e("CHECK_IMPEQK", 8, 0, 4, 1, 2, imm=0x10000)],
        "N_ADD": [e("N_ADD", 8, 5, 0, 1)],
        "N_EQN": [e("N_EQN", 1, 5, 0, 1)],
        "MOV_N": [e("MOV_N", 8, 5, 1)],
        "N_EQ_wide": [e("N_EQ", 256, 5, 0, 1)],
        "W_ADD": [e("W_ADD", 256, 2, 0, 1)],
        "W_AND": [e("W_AND", 256, 2, 0, 1)],
        "LEAF_N": [e("LEAF_N", 8, 5, imm=idx["n0"])],
        "LEAF_W": [e("LEAF_W", 256, 2, imm=idx["w0"])],
        # one guarded calldata byte (index 0x24 < size w1) into W2, unchained
        "W_CDINS": [e("W_CDINS", 256, 2, 2, 1, kw(p, 0x24), imm=idx["n0"] | (8 << 16))],
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--repeat", type=int, default=2000)
    ap.add_argument("--log2", type=int, default=20)
    ap.add_argument("--only", default=None)
    ap.add_argument("--engines", default="asm,interp")
    a = ap.parse_args()
    from mythril_amd.runtime import Device
    dev = Device(0)
    n = 1 << a.log2
    slots = 256 * 4 * 2   # CUs x SIMDs x waves per SIMD
    cases = [(p, name + suffix, body)
             for p, suffix in ((base_program(False), ""), (base_program(True), "_pool"))
             for name, body in variants(p).items()]
    for p, name, body in cases:
        if a.only and name != a.only:
            continue
        # leaf-drawing instructions cost several dispatches: fewer repeats
        rep = a.repeat // 4 if name.startswith(("LEAF", "W_CDINS")) else a.repeat
        q = assemble(p, body, rep)
        dp = dev.load(q)
        # asm: the threaded-dispatch interpreter (default); interp: the compiled
        # one (MYTHRIL_AMD_ASM=0, read by the library at each call).  Two
        # launches each (warm-up, measured): tools/opcost_summary.py pairs the
        # PMC rows with these lines in order.
        for engine in a.engines.split(","):
            os.environ["MYTHRIL_AMD_ASM"] = "0" if engine == "interp" else "1"
            ran = dev.engine_of(dp)
            dev.search([dp], 1, 0, n, 0)   # warm
            _, st = dev.search([dp], 1, 0, n, 0)
            waves = n // 64
            ns_per = st["kernel_ms"] * 1e6 / (waves / slots) / rep
            print(json.dumps({"op": name, "engine": ran, "repeat": rep, "log2": a.log2,
                              "kernel_ms": round(st["kernel_ms"], 3),
                              "ns_per_insn_per_wave_slot": round(ns_per, 1),
                              "cycles_at_2p4GHz": round(ns_per * 2.4, 0)}), flush=True)
        dp.free()
    dev.close()


if __name__ == "__main__":
    main()
