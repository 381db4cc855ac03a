"""The LaserEVM-order replay of tests/test_laser_replay.py on the MI355X with
the drop-in's default candidate budget (2^22): one search launch per JUMPI
pair (and per transaction-boundary prefetch), and every
device witness confirmed by the oracle's re-check.  Prints one record per
scenario (launches per query, memo hits, Keccak requests) for DESIGN.md."""
import json

import pytest

from tests.test_laser_replay import RUNS, replay

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def device():
    from mythril_amd.runtime import Device
    d = Device(0)
    yield d
    d.close()


@pytest.mark.parametrize("name", sorted(RUNS))
def test_replay_on_device(name, monkeypatch, device):
    from mythril_amd.engine import DEFAULT_BUDGET
    answers, expect, rec = replay(name, monkeypatch, device, DEFAULT_BUDGET)
    rec["launches_per_query"] = rec["launches"] / rec["is_possible"]
    print("LASER replay", name, json.dumps(rec))
    m, run, _ = RUNS[name]
    for q, got, exp in zip(run.queries, answers, expect):
        if q.sat or exp:
            assert got, q.pc
    # one launch per JUMPI pair, plus one per transaction-boundary prefetch and
    # per detection-module query
    assert rec["launches"] * 2 <= rec["jumpi_prunes"] + 1 + 2 * rec["tx_prunes"] + 2 * rec["module_queries"]
    assert rec["z3_confirmed"] == rec["gpu_witnesses"]
