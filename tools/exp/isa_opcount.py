#!/usr/bin/env python3
"""Static gfx950 instruction counts per DAG op in the specialised kernels (CPU only).

For each op class, a chain of N dependent ops (tools/opbench.py's chain) is
compiled by jit.py and disassembled; prints VALU / v_mov / s_nop / SALU /
v_mad_u64_u32 counts per op.  Used to pick ALU rewrites before spending GPU time.

Usage: python tools/exp/isa_opcount.py [N] [op ...]
"""
import collections
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from mythril_amd import jit  # noqa: E402
from mythril_amd.compiler import compile_program  # noqa: E402
from opbench import OPS, chain  # noqa: E402

LLVM = "/opt/rocm/lib/llvm/bin"


def disasm(image: bytes) -> list:
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "k.hsaco")
        co = os.path.join(td, "k.co")
        open(src, "wb").write(image)
        subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={src}",
                               "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"])
        txt = subprocess.check_output([f"{LLVM}/llvm-objdump", "-d", co], text=True)
    return [ln.split("//")[0].strip() for ln in txt.splitlines() if ln.startswith("\t")]


def classify(ins: list) -> collections.Counter:
    c = collections.Counter()
    for i in ins:
        op = i.split()[0] if i else ""
        if op.startswith("v_"):
            c["valu"] += 1
            if op.startswith("v_mov_b32"):
                c["v_mov"] += 1
            if op.startswith("v_cndmask"):
                c["cndmask"] += 1
            if op == "v_mad_u64_u32":
                c["mad64"] += 1
            if op.startswith(("v_mul_lo", "v_mul_hi")):
                c["mul32"] += 1
            if op.startswith(("v_addc", "v_subb", "v_add_co", "v_sub_co", "v_subrev_co", "v_subbrev")):
                c["carry"] += 1
        elif op == "s_nop":
            c["s_nop"] += 1
            c["nop_states"] += int(i.split()[1]) + 1
        elif op.startswith("s_"):
            c["salu"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
    return c


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    ops = sys.argv[2:] or OPS
    # baseline: the same kernel shell with a 1-op chain, subtracted out
    keys = ["valu", "v_mov", "s_nop", "nop_states", "salu", "mad64", "mul32", "carry", "cndmask", "lds"]
    print(f"{'op':8s} " + " ".join(f"{k:>9s}" for k in keys) + "   (per op)")
    for op in ops:
        nn = n // 8 if op in ("bvudiv", "bvurem") else n
        cnt = []
        for m in (1, nn + 1):
            c, conj = chain(op, n=m)
            p = compile_program(conj)
            image, names, _ = jit.compile_device([p], "x", fence_first=True)
            cnt.append(classify(disasm(image)))
        d = {k: (cnt[1][k] - cnt[0][k]) / nn for k in keys}
        print(f"{op:8s} " + " ".join(f"{d[k]:9.1f}" for k in keys), flush=True)


if __name__ == "__main__":
    main()
