"""bench.py --gpus N: without a torchrun environment the
script starts N rank processes itself, and every rank searches its own slice.
Here on CPU: 2 ranks over gloo with the host build of the interpreter standing
in for the device; the reported witness (all-reduce MIN over ranks) and the
time-to-first-witness index (per-slice MIN, cross-rank early stop) must equal a
single-process search of the same ranges."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODES = 200
WITNESS = 0x5EED0005 % (1 << 31)      # synth.build_c5's planted index
BATCH_LOG2 = 8


def _single_process_min(begin, count):
    from mythril_amd.compiler import compile_program
    from mythril_amd.hostemu import term_values
    from mythril_amd.synth import build_c5
    from tests.fakedev import FakeDevice
    syn = build_c5(term_values, n_nodes=NODES)
    dev = FakeDevice(chunk=1 << 12)
    (found,), _ = dev.search([dev.load(compile_program(syn.conjuncts))], syn.seed, begin, count, 0)
    return found


def _run_bench(extra):
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--host-emulator", "--dist-backend", "gloo",
           "--engine", "interp", "--nodes", str(NODES), "--batch-log2", str(BATCH_LOG2), "--steps", "1",
           "--warmup", "0", "--no-cpu-baseline"] + extra
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout     # one JSON line, from rank 0 only
    return json.loads(lines[0])


def test_bench_spawns_two_ranks_and_reduces_the_minimum():
    begin = WITNESS - 300                # the planted witness falls in rank 1's slice
    out = _run_bench(["--gpus", "2", "--begin", str(begin), "--ttfw-slice-log2", "8",
                      "--ttfw-max-slices", "4", "--ttfw-begin", str(WITNESS - 700)])
    assert out["n_gpus"] == 2
    assert out["config"]["rccl_world"] == 2
    assert out["config"]["dist_backend"] == "gloo"
    single = _single_process_min(begin, 2 << BATCH_LOG2)
    assert single is not None
    assert out["config"]["witness_found_in_timed_range"] == single
    # TTFW: slices of 2 x 256 from WITNESS-700; the first hit is in slice 1
    ttfw = out["config"]["time_to_first_witness"]
    assert ttfw["index"] == _single_process_min(WITNESS - 700, 4 * (2 << 8))
    assert ttfw["candidates_searched"] == 2 * (2 << 8)
    assert out["value"] > 0 and out["scaling"] == "weak"


def test_bench_rejects_mismatched_world_size():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_bench_rejects_devices_with_ranks():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--devices", "2"], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "exclude" in r.stderr
