"""bench.py's roofline side inputs (CPU): the committed PMC traffic is found for
the kernel the benchmark attaches (its module name, without the launched
symbol's _x suffix), and the measured VALU peak loads."""
import json
import os

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class _Prog:
    def __init__(self, ops):
        self.ops_per_eval = ops


def test_traffic_found_for_attached_kernel_name():
    d = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    kernel = d["kernel_name"]
    assert kernel.endswith("_x")
    module = kernel[:-2]                      # what jit.attach records as dp.kernel
    prog = _Prog(d["ops_per_eval"])
    assert bench.load_traffic(prog, d["batch"], module) == d["hbm_bytes_per_launch"]
    assert bench.load_traffic(prog, d["batch"], kernel) == d["hbm_bytes_per_launch"]
    assert bench.load_traffic(prog, d["batch"], module[:-1]) is None     # another kernel
    assert bench.load_traffic(prog, d["batch"] * 2, module) is None      # another batch
    assert bench.load_traffic(_Prog(d["ops_per_eval"] + 1), d["batch"], module) is None


def test_measured_peak_loads():
    peak = bench.load_measured_peak()
    assert peak is not None and 0.5 * bench.THEORETICAL_PEAK < peak <= bench.THEORETICAL_PEAK
