"""WalletLibrary-shaped Keccak at LaserEVM's batch sites (VERDICT r5 item 7;
``WalletLibrary.sol:389-397``: ``mapping(uint => uint) m_ownerIndex``,
``mapping(bytes32 => PendingState) m_pending``; the fixtures' own mapping
contracts ``underflow`` (token.sol), ``overflow`` and ``metacoin`` have the
same ``mapping(address => uint) balances`` shape).

Replayed in LASER's order (tests/laser_replay.py) with the plugin's Keccak
speculation on (``MYTHRIL_AMD_KECCAK_SPECULATION=1``) and the product's
device threshold (``KeccakService.min_batch`` 64), every batch the service
sees is recorded:

* at each ``stop_sym_trans`` the mapping-entry preimages ``pad32(key) ++
  pad32(slot)`` of LASER's three actors and the target contract, and the
  array bases ``pad32(slot)``, for slots 0-15 (``prefetch_storage_slots``);
* the report-time batch ``_replace_with_actual_sha`` /
  ``get_concrete_hash_data`` hashes: the concrete preimages of every
  ``keccak256_512`` point in the device witnesses of the detection modules'
  queries (``sender_N ++ slot``, ``keccak_function_manager.py:95-114``);
* the concrete SHA3 requests the transactions make (``find_concrete_keccak``,
  ``keccak_function_manager.py:57-69``), and how many the memo answers.

``keccak_batches`` returns the record; the CPU test runs it on the host build
of the Keccak kernel, tests/test_gpu_keccak_batches.py on the device, where
every digest a device batch produced equals oracle/keccak."""
import pytest

from mythril_amd import keccak_service, mythril_plugin
from mythril_amd import model as dropin
from mythril_amd import z3bridge
from mythril_amd.engine import WitnessEngine
from oracle.dag_eval import eval_nodes
from oracle.keccak import keccak256
from tests.fakedev import FakeDevice
from tests.laser_replay import ReplayVM, install_standins
from tests.test_laser_replay import RUNS

MAPPING_RUNS = ["underflow/t3_send_send_balance", "overflow/t3_send_send_balance", "metacoin/t3_sendtoken"]


def keccak_batches(name, monkeypatch, dev, budget):
    m, run, ntx = RUNS[name]

    def model_for(nodes):
        vals = eval_nodes(nodes, run.model)
        return run.model if all(vals[n.id] for n in nodes) else None

    install_standins(monkeypatch, model_for, m.c)
    witnesses = []
    confirm = z3bridge.model_from_witness

    def recording_confirm(raws, script, w, timeout_ms=2000):
        witnesses.append(w)
        return confirm(raws, script, w, timeout_ms)
    monkeypatch.setattr(z3bridge, "model_from_witness", recording_confirm)
    monkeypatch.setattr(dropin, "_engine", WitnessEngine(dev=dev, budget=budget))
    monkeypatch.setattr(dropin, "_engine_failed", False)
    monkeypatch.setattr(dropin, "_reference", None)
    dropin._memo.clear()
    dropin._misses.clear()
    dropin._pending.clear()
    dropin.get_model.cache_clear()
    svc = keccak_service.KeccakService(device=dev, reference=lambda b: keccak256(b))   # the product's threshold
    monkeypatch.setattr(keccak_service, "_service", svc)
    monkeypatch.setattr(keccak_service, "install", lambda device=None: False)
    monkeypatch.setattr(mythril_plugin, "KECCAK_SPECULATION", True)
    vm = ReplayVM()
    mythril_plugin.MI355XWitnessEngine()().initialize(vm)
    requests = []

    def concrete(value, bits):
        before = svc.stats["memo_hits"]
        d = svc.find_concrete_keccak_int(value, bits)
        requests.append(svc.stats["memo_hits"] > before)
        return d
    vm.replay([(run, ntx)], keccak=concrete)
    speculation = list(svc.batches)
    # the report-time batch: the preimages of the keccak256_512 points the
    # device witnesses carry (what _replace_with_actual_sha hashes)
    pre = sorted({(512, args[0]) for w in witnesses for f, table in w.functions.items()
                  if f.startswith("keccak256_512") and "-1" not in f for args in table})
    svc.prefetch_values(pre)
    report = svc.batches[len(speculation):]
    rec = {"run": name, "transactions": ntx, "min_batch": svc.min_batch,
           "speculation_batches": speculation, "report_batches": report,
           "report_preimages": len(pre), "concrete_requests": len(requests),
           "concrete_memo_hits": sum(requests), "stats": dict(svc.stats)}
    return rec, svc


def check_digests(svc):
    """Every digest in the memo (device batches included) is the oracle's."""
    for msg, d in svc.memo.items():
        assert d == keccak256(msg), msg.hex()


@pytest.mark.parametrize("name", MAPPING_RUNS)
def test_mapping_keccak_batches(name, monkeypatch):
    dev = FakeDevice(chunk=1 << 10)
    rec, svc = keccak_batches(name, monkeypatch, dev, 1 << 12)
    print("keccak batches", rec)
    # one speculation batch per stop_sym_trans: 4 keys (3 actors, the target)
    # x 16 slots + 16 array bases = 80 preimages, past the device threshold
    spec = rec["speculation_batches"]
    assert len(spec) == rec["transactions"] and spec[0]["size"] == 80 and spec[0]["device"]
    assert all(b["new"] == 0 for b in spec[1:])          # the same keys: memo hits
    assert getattr(dev, "keccak_launches", 0) >= 1
    check_digests(svc)
