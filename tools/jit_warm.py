#!/usr/bin/env python3
"""Pre-compile the specialised kernels bench.py, the GPU tests and (with
--opbench) tools/opbench.py use into the in-tree JIT cache (build/jit), so GPU
runs do not spend minutes in hipcc; --prune then deletes every other cache
entry (the cache travels with each GPU run).  __graft_entry__.build() runs it."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    """Every compile is an independent hipcc process: run them on a thread pool
    (the C5 kernel alone takes ~8 minutes; sequentially the warm-up took ~24)."""
    import time
    from concurrent.futures import ThreadPoolExecutor
    from mythril_amd import jit
    from mythril_amd.compiler import compile_program
    t0 = time.perf_counter()
    jobs = list(jit.bench_warm_jobs())   # longest first

    def gpu_jit_modules():
        from tests.helpers import division_check_programs
        from tests.test_gpu_jit import small_planted
        from tests.test_jit import _random_programs
        planted = [small_planted(n_nodes=300, n_conj=6, density_log2=8 + k, seed=0x5EED0005 + k) for k in range(3)]
        progs = [compile_program(s.conjuncts) for s in planted] + [p for *_, p in _random_programs(8, 9100)] + \
            division_check_programs()
        print("tests/test_gpu_jit.py module:", jit.compile_device(progs)[2], "s", flush=True)
        print("tests/test_gpu_jit.py LDS module:", jit.compile_device(progs[:11], lds_leaves=4)[2], "s", flush=True)
        for p in progs[:2]:
            print("tests/test_gpu_jit.py parts:", jit.compile_parts(p, lds_leaves=2, part_weight=3000)[1], "s",
                  flush=True)

    def constant_divisors():
        from tests.helpers import constant_divisor_programs
        print("tests/test_gpu_jit.py constant divisors:", jit.compile_device(constant_divisor_programs())[2], "s",
              flush=True)

    def mul_cols():
        from tests.helpers import mul_check_programs
        for cols in (True, False):
            print("tests/test_gpu_jit.py mul_cols=%s:" % cols,
                  jit.compile_device(mul_check_programs(), mul_cols=cols)[2], "s", flush=True)

    from config_bench import warm_jobs as config_jobs   # tools/config_bench.py (C2-C4 solver-log queries)
    jobs += config_jobs() + [gpu_jit_modules, constant_divisors, mul_cols]
    if "--opbench" in sys.argv:
        from opbench import OPS, chain

        def opbench(op):
            c, conj = chain(op, n=50 if op in ("bvudiv", "bvurem") else 400)
            print(op, jit.compile_device([compile_program(conj)], "x", fence_first=True)[2], "s", flush=True)
        jobs += [(lambda op=op: opbench(op)) for op in OPS]
    workers = max(1, min(len(jobs), int(os.environ.get("MW_JIT_JOBS", str(os.cpu_count() or 8)))))
    with ThreadPoolExecutor(workers) as ex:
        for f in [ex.submit(j) for j in jobs]:
            f.result()   # re-raise the first failure
    print(f"jit warm-up: {len(jobs)} jobs on {workers} workers in {time.perf_counter() - t0:.0f} s", flush=True)
    if "--prune" in sys.argv:
        print("pruned", jit.prune_cache(), "stale cache entries", flush=True)


if __name__ == "__main__":
    main()
