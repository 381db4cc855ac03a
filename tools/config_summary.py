#!/usr/bin/env python3
"""One line per (config, engine) of tools/config_bench.py's JSON output(s):
evals/s, the fraction of the guide peak on the smaller of the DAG-priced and
instruction-priced op counts (frac), both counts, and the DAG-priced fraction.

    python tools/config_summary.py gpurun_out/TAG/config_bench.json [...]
"""
import json
import sys

for path in sys.argv[1:]:
    for ln in json.load(open(path)):
        print(f"{path.split('/')[-2]:8s} {ln['config']:4s} {ln['engine'].split()[0]:7s} {str(ln['kernels']):10s} "
              f"{ln['evals_per_s'] / 1e9:8.3f} G evals/s  kernel {ln['kernel_ms']:9.2f} ms  frac {ln['frac_peak']:.3f}"
              f"  ops {ln['ops_per_eval']} executed {ln.get('executed_ops_per_eval', ln['ops_per_eval'])}"
              f"  frac_nominal {ln.get('frac_peak_nominal', ln['frac_peak']):.3f}")
