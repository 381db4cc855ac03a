#!/usr/bin/env python3
"""Experiment: where the per-candidate fixed cost of the
Mythril-shaped queries goes.  Builds the interpreter library and the C2/C2L/C4
specialised kernels with one part of candidate generation replaced by a cheap
stand-in (csrc/mw_leaf.h MW_ABLATE_*: wrong values, same data flow), then
times tools/config_bench.py on each variant.

    python tools/leaf_ablate.py --build            # CPU: libraries + JIT cache
    python tools/leaf_ablate.py --run OUTDIR       # GPU box: one config_bench per variant
"""
import argparse
import json
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VARIANTS = {"base": [], "leaf": ["-DMW_ABLATE_LEAF"], "philox": ["-DMW_ABLATE_PHILOX"],
            "digit": ["-DMW_ABLATE_DIGIT"]}
ONLY = "C2,C2L,C4"


def lib_path(v):
    return os.path.join(ROOT, "build", "ab", v, "libmythril_witness.so")


def build():
    from mythril_amd.build import CSRC, DEVICE_SRCS, _hipcc
    jobs = []
    for v, flags in VARIANTS.items():
        if v == "base":
            continue
        os.makedirs(os.path.dirname(lib_path(v)), exist_ok=True)
        jobs.append([_hipcc(), "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", *flags,
                     "-Wno-unused-result", "-Wno-unused-value", *DEVICE_SRCS, "-o", lib_path(v)])
    with ThreadPoolExecutor(4) as ex:
        for r in ex.map(lambda c: subprocess.run([str(x) for x in c], cwd=CSRC), jobs):
            assert r.returncode == 0
    for v, flags in VARIANTS.items():
        env = dict(os.environ, MYTHRIL_AMD_JIT_FLAGS=" ".join(flags))
        code = ("import sys; sys.path.insert(0, 'tools'); from config_bench import warm_jobs, CONFIGS; "
                "from concurrent.futures import ThreadPoolExecutor; import config_bench; "
                f"config_bench.CONFIGS = [c for c in CONFIGS if c[0] in {ONLY.split(',')!r}]; "
                "jobs = warm_jobs(); ex = ThreadPoolExecutor(8); [f.result() for f in [ex.submit(j) for j in jobs]]")
        subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, check=True)
        print("warmed", v, flush=True)


def run(outdir):
    os.makedirs(outdir, exist_ok=True)
    summary = {}
    for v, flags in VARIANTS.items():
        env = dict(os.environ, MYTHRIL_AMD_JIT_FLAGS=" ".join(flags))
        if v != "base":
            env["MYTHRIL_AMD_LIB"] = lib_path(v)
        out = os.path.join(outdir, f"ablate_{v}.json")
        subprocess.run(["timeout", "-k", "10", "280", sys.executable, "tools/config_bench.py", "--only", ONLY,
                        "--out", out], cwd=ROOT, env=env, check=True)
        summary[v] = {f"{ln['config']} {ln['engine'].split()[0]}": ln["evals_per_s"] for ln in json.load(open(out))}
    print(json.dumps(summary, indent=1))
    json.dump(summary, open(os.path.join(outdir, "ablate_summary.json"), "w"), indent=1)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--run", default=None)
    a = ap.parse_args()
    if a.build:
        build()
    if a.run:
        run(a.run)
