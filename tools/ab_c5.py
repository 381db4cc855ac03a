#!/usr/bin/env python3
"""Experiment: A/B of C5 specialised-kernel code generation variants on one GPU.

Variants are jit.py settings (asm pass on/off); each is compiled into the
in-tree cache (run with --compile-only on the CPU first), attached to the same
loaded C5 program, timed over 2^22-candidate exhaustive launches, and checked
to give the same witness and candidate count as the first variant.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from mythril_amd import hostemu, jit  # noqa: E402
from mythril_amd.compiler import compile_program  # noqa: E402
from mythril_amd.synth import build_c5  # noqa: E402

VARIANTS = {"base": {"EXTRA_FLAGS": []},
            # ablations (wrong results, timing only): one op class replaced by an XOR
            "abl_mul": {"EXTRA_FLAGS": ["-DMW_ABLATE_MUL"]}, "abl_div": {"EXTRA_FLAGS": ["-DMW_ABLATE_DIV"]},
            "abl_add": {"EXTRA_FLAGS": ["-DMW_ABLATE_ADD"]}, "abl_shift": {"EXTRA_FLAGS": ["-DMW_ABLATE_SHIFT"]},
            # code generation: two conjunct chains merged per basic block (jit.interleave_conjuncts)
            "il2": {"EXTRA_FLAGS": [], "interleave": 2},
            "abl_knuth": {"EXTRA_FLAGS": ["-DMW_ABLATE_KNUTH"]}, "abl_fulldiv": {"EXTRA_FLAGS": ["-DMW_ABLATE_FULLDIV"]},
            # one wave per SIMD: 512 registers per lane, no leaves in LDS
            "w1": {"EXTRA_FLAGS": [], "waves": 1, "lds": 0},
            # a workgroup barrier after every conjunct (jit.CHECK_SYNC): the block's waves fetch the same code
            "sync": {"EXTRA_FLAGS": [], "CHECK_SYNC": True},
            # the division's rare paths without branch weights (in line, as before round 3)
            "nohint": {"EXTRA_FLAGS": ["-DMW_DIV_NO_HINTS"]},
            # round 4's smaller division code, measured slower (profiles/r4h): the short
            # division's steps as a rolled loop, the limb-aligned path's limb shifts as one
            "shortroll": {"EXTRA_FLAGS": ["-DMW_SHORT_ROLLED"]},
            "genroll": {"EXTRA_FLAGS": ["-DMW_GEN_ROLLED_SHIFT"]},
            "r4roll": {"EXTRA_FLAGS": ["-DMW_SHORT_ROLLED", "-DMW_GEN_ROLLED_SHIFT"]},
            # three waves per SIMD (170 registers per lane); LDS leaves cost 8 KiB per slot and
            # block, so 3 blocks per CU (160 KiB) allow at most 6
            "w3": {"EXTRA_FLAGS": [], "waves": 3, "lds": 6}, "w3l0": {"EXTRA_FLAGS": [], "waves": 3, "lds": 0},
            # two waves per SIMD with fewer / more leaves in LDS than the default 10
            "l6": {"EXTRA_FLAGS": [], "lds": 6}, "l8": {"EXTRA_FLAGS": [], "lds": 8},
            "l12": {"EXTRA_FLAGS": [], "lds": 12},
            # LLVM scheduler choices
            "ilp": {"EXTRA_FLAGS": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]},
            "bias0": {"EXTRA_FLAGS": ["-mllvm", "-amdgpu-schedule-metric-bias=0"]},
            "trackers": {"EXTRA_FLAGS": ["-mllvm", "-amdgpu-use-amdgpu-trackers"]},
            # optimisation levels that trade instructions for code size (instruction-fetch wait)
            "os": {"EXTRA_FLAGS": ["-Os"]}, "o2": {"EXTRA_FLAGS": ["-O2"]},
            # 256-bit products by columns with v_mad_u64_u32 carry-outs (mw_jit.h mul8_cols)
            "mulcols": {"EXTRA_FLAGS": [], "MUL_COLS": True}, "rows": {"EXTRA_FLAGS": [], "MUL_COLS": False},
            # LDS leaf reloads placed k body lines ahead of their use (jit.LDS_AHEAD)
            "ahead8": {"EXTRA_FLAGS": [], "LDS_AHEAD": 8}, "ahead16": {"EXTRA_FLAGS": [], "LDS_AHEAD": 16},
            "ahead32": {"EXTRA_FLAGS": [], "LDS_AHEAD": 32}, "ahead64": {"EXTRA_FLAGS": [], "LDS_AHEAD": 64},
            "a32l12": {"EXTRA_FLAGS": [], "LDS_AHEAD": 32, "lds": 12},
            "a32l14": {"EXTRA_FLAGS": [], "LDS_AHEAD": 32, "lds": 14},
            "a32l8": {"EXTRA_FLAGS": [], "LDS_AHEAD": 32, "lds": 8},
            # ... by estimated work instead of lines (jit.LDS_AHEAD_W)
            "w60": {"EXTRA_FLAGS": [], "LDS_AHEAD_W": 60}, "w120": {"EXTRA_FLAGS": [], "LDS_AHEAD_W": 120},
            "w240": {"EXTRA_FLAGS": [], "LDS_AHEAD_W": 240}, "w480": {"EXTRA_FLAGS": [], "LDS_AHEAD_W": 480},
            # ... not above a division (jit.LDS_AHEAD_STOP)
            "a8s": {"EXTRA_FLAGS": [], "LDS_AHEAD": 8, "LDS_AHEAD_STOP": 500},
            "a16s": {"EXTRA_FLAGS": [], "LDS_AHEAD": 16, "LDS_AHEAD_STOP": 500},
            "a8m": {"EXTRA_FLAGS": [], "LDS_AHEAD": 8, "LDS_AHEAD_STOP": 100},
            "a4": {"EXTRA_FLAGS": [], "LDS_AHEAD": 4},
            "a32s": {"EXTRA_FLAGS": [], "LDS_AHEAD": 32, "LDS_AHEAD_STOP": 500},
            # basic-block length of the straight-line body (jit.SPLIT_EVERY, default 48)
            "sp32": {"EXTRA_FLAGS": [], "SPLIT_EVERY": 32}, "sp64": {"EXTRA_FLAGS": [], "SPLIT_EVERY": 64},
            "sp96": {"EXTRA_FLAGS": [], "SPLIT_EVERY": 96}, "sp128": {"EXTRA_FLAGS": [], "SPLIT_EVERY": 128},
            "sp192": {"EXTRA_FLAGS": [], "SPLIT_EVERY": 192}, "sp256": {"EXTRA_FLAGS": [], "SPLIT_EVERY": 256},
            # a workgroup barrier after every k-th conjunct (the block's waves fetch the same code)
            "sync8": {"EXTRA_FLAGS": [], "CHECK_SYNC": True, "CHECK_SYNC_EVERY": 8},
            "sync32": {"EXTRA_FLAGS": [], "CHECK_SYNC": True, "CHECK_SYNC_EVERY": 32},
            "sync128": {"EXTRA_FLAGS": [], "CHECK_SYNC": True, "CHECK_SYNC_EVERY": 128},
            # a leaf's recent LDS reload read again instead of reloading (jit.LDS_REUSE)
            "reuse4": {"EXTRA_FLAGS": [], "LDS_REUSE": 4}, "reuse12": {"EXTRA_FLAGS": [], "LDS_REUSE": 12},
            "reuse24": {"EXTRA_FLAGS": [], "LDS_REUSE": 24}, "reuse48": {"EXTRA_FLAGS": [], "LDS_REUSE": 48},
            "reuse96": {"EXTRA_FLAGS": [], "LDS_REUSE": 96}, "reuse192": {"EXTRA_FLAGS": [], "LDS_REUSE": 192},
            "reuse128": {"EXTRA_FLAGS": [], "LDS_REUSE": 128},
            "l8r96": {"EXTRA_FLAGS": [], "LDS_REUSE": 96, "lds": 8},
            "a32r96": {"EXTRA_FLAGS": [], "LDS_REUSE": 96, "LDS_AHEAD": 32}}


MUL_COLS_DEFAULT = jit.MUL_COLS
LDS_AHEAD_DEFAULT = jit.LDS_AHEAD
LDS_AHEAD_W_DEFAULT = jit.LDS_AHEAD_W
LDS_AHEAD_STOP_DEFAULT = jit.LDS_AHEAD_STOP
SPLIT_EVERY_DEFAULT = jit.SPLIT_EVERY
LDS_REUSE_DEFAULT = jit.LDS_REUSE


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--compile-only", action="store_true")
    ap.add_argument("--variants", default="base")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=1)
    ap.add_argument("--out", default="gpurun_out/ab_c5.json")
    a = ap.parse_args()
    syn = build_c5(hostemu.term_values)
    p = compile_program(syn.conjuncts)
    images = {}
    for v in a.variants.split(","):
        opts = {"CHECK_SYNC": False, "CHECK_SYNC_EVERY": 1, "LDS_REUSE": LDS_REUSE_DEFAULT, "MUL_COLS": MUL_COLS_DEFAULT, "LDS_AHEAD": LDS_AHEAD_DEFAULT, "LDS_AHEAD_W": LDS_AHEAD_W_DEFAULT,
                "LDS_AHEAD_STOP": LDS_AHEAD_STOP_DEFAULT, "SPLIT_EVERY": SPLIT_EVERY_DEFAULT, **VARIANTS[v]}
        il = opts.pop("interleave", 1)
        waves, lds = opts.pop("waves", 2), opts.pop("lds", 10)
        for k, val in opts.items():
            setattr(jit, k, val)
        image, names, dt = jit.compile_device([p], "x", waves=waves, lds_leaves=lds, interleave=il)
        images[v] = (image, names[0])
        print(f"{v}: {names[0]} {len(image)} B {'compiled in %.0f s' % dt if dt else 'cached'}", flush=True)
    if a.compile_only:
        return
    from mythril_amd.runtime import Device
    dev = Device(0)
    res = {}
    w = syn.witness_index
    for rnd in range(a.rounds):          # variants alternate: box drift lands on all of them
        for v, (image, name) in images.items():
            dp = dev.load(p)
            dev.attach_kernel(dp, image, name)
            dev.search([dp], syn.seed, 0, 1 << 22)  # warm
            ms = []
            for _ in range(a.reps):
                _, st = dev.search([dp], syn.seed, 0, 1 << 22)
                ms.append(st["kernel_ms"])
            (hit,), st = dev.search([dp], syn.seed, w - (1 << 20), (1 << 20) + 1)
            r = res.setdefault(v, {"all_ms": [], "witness": hit, "evals": st.get("evals")})
            r["all_ms"] += ms
            r["kernel_ms"] = sorted(r["all_ms"])[len(r["all_ms"]) // 2]
            assert r["witness"] == hit, (v, hit)
            print(v, rnd, json.dumps({"kernel_ms": sorted(ms)[len(ms) // 2], "witness": hit}), flush=True)
            dp.free()
    res["planted"] = w
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
