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
    from mythril_amd import jit
    jit.warm_bench_cache()
    from mythril_amd.compiler import compile_program
    from tests.helpers import division_check_programs
    from tests.test_gpu_jit import small_planted
    from tests.test_jit import _random_programs
    planted = [small_planted(n_nodes=300, n_conj=6, density_log2=8 + k, seed=0x5EED0005 + k) for k in range(3)]
    progs = [compile_program(s.conjuncts) for s in planted] + [p for *_, p in _random_programs(8, 9100)] + \
        division_check_programs()
    print("tests/test_gpu_jit.py module:", jit.compile_device(progs)[2], "s", flush=True)
    print("tests/test_gpu_jit.py LDS module:", jit.compile_device(progs[:11], lds_leaves=4)[2], "s", flush=True)
    for p in progs[:2]:
        print("tests/test_gpu_jit.py parts:", jit.compile_parts(p, lds_leaves=2, part_weight=3000)[1], "s", flush=True)
    from tests.helpers import constant_divisor_programs
    print("tests/test_gpu_jit.py constant divisors:", jit.compile_device(constant_divisor_programs())[2], "s",
          flush=True)
    from config_bench import warm as warm_configs
    warm_configs()   # tools/config_bench.py (C2-C4 solver-log queries)
    print("tools/config_bench.py kernels warmed", flush=True)
    if "--opbench" in sys.argv:
        from opbench import OPS, chain
        for op in OPS:
            c, conj = chain(op, n=50 if op in ("bvudiv", "bvurem") else 400)
            print(op, jit.compile_device([compile_program(conj)], "x", fence_first=True)[2], "s", flush=True)
    if "--prune" in sys.argv:
        print("pruned", jit.prune_cache(), "stale cache entries", flush=True)


if __name__ == "__main__":
    main()
