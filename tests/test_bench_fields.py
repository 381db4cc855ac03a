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


def test_cpu_baseline_checks_verdicts_around_the_planted_witness():
    """The CPU leg's samples from index 0 hold no satisfying candidate, so it
    also compares the verdicts of the candidates around the planted witness:
    the host build, the C oracle and the (emulated) device agree there and
    each finds the witness (host emulator: plumbing, not a measurement)."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--host-emulator", "--engine", "interp",
                        "--nodes", "300", "--batch-log2", "12", "--steps", "1", "--warmup", "0",
                        "--cpu-seconds", "0.5", "--no-ttfw"], cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    win = out["cpu_baseline"]["witness_window"]
    assert win["count"] == 8192 and win["begin"] <= 0x5EED0005 % (1 << 31) < win["begin"] + win["count"]
    assert win["satisfied_gpu"] >= 1
    for leg in ("host_build", "oracle"):
        assert win[f"satisfied_{leg}"] == win["satisfied_gpu"]
        assert win[f"mismatches_{leg}_vs_gpu"] == 0
