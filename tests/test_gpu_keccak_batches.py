"""tests/test_keccak_batches.py on the MI355X: the
WalletLibrary-shaped mapping runs replayed in LASER's order with the Keccak
speculation on; the speculation batch crosses the device threshold and is
hashed by the batched Keccak-256 kernel, and every digest the device produced
equals oracle/keccak.  Prints one record per run for DESIGN.md."""
import json

import pytest

from tests.test_keccak_batches import MAPPING_RUNS, check_digests, keccak_batches

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def device():
    from mythril_amd.runtime import Device
    d = Device(0)
    yield d
    d.close()


@pytest.mark.parametrize("name", MAPPING_RUNS)
def test_mapping_keccak_batches_on_device(name, monkeypatch, device):
    from mythril_amd.engine import DEFAULT_BUDGET
    rec, svc = keccak_batches(name, monkeypatch, device, DEFAULT_BUDGET)
    print("keccak batches", json.dumps(rec))
    assert rec["stats"]["launches"] >= 1 and rec["stats"]["gpu_hashes"] >= svc.min_batch
    assert any(b["device"] for b in rec["speculation_batches"])
    check_digests(svc)
