"""The drop-in get_model (tests/test_dropin.py's stand-in Mythril) with the
witness engine on the MI355X: feasible queries answered by the device and
confirmed, UNSAT ones falling back to the reference, and the batched
transaction-boundary prefetch (svm.py:216-223) feeding the memo."""
import pytest

from mythril_amd import model as dropin
from tests.test_dropin import CTX, SAT, UNSAT, UnsatError, X, fb, mythril  # noqa: F401 (fixture)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def device():
    from mythril_amd.runtime import Device
    d = Device(0)
    yield d
    d.close()


@pytest.fixture
def on_gpu(mythril, monkeypatch, device):  # noqa: F811
    from mythril_amd.engine import WitnessEngine
    monkeypatch.setattr(dropin, "_engine", WitnessEngine(dev=device, budget=1 << 16))
    return mythril


def test_feasible_query_answered_on_device(on_gpu):
    res = dropin.get_model(SAT)
    assert res.raw[0][0] == "z3" and 200 < res.raw[0][1]["x"] < 203
    assert on_gpu.calls["reference"] == 0
    assert dropin._engine.stats["searches"] >= 1 and dropin._engine.stats["hits"] >= 1


def test_unsat_falls_back_on_device(on_gpu):
    with pytest.raises(UnsatError):
        dropin.get_model(UNSAT)
    assert on_gpu.calls["reference"] == 1


def test_prefetch_one_launch_on_device(on_gpu):
    sets = [SAT, (fb(CTX.app("=", X, CTX.const(77, 8))),), UNSAT]
    assert dropin.prefetch(sets) == 2
    n = dropin._engine.stats["searches"]
    assert n == 1  # all three sets in one mg_search
    assert dropin.get_model(sets[1]).raw[0][1]["x"] == 77
    assert dropin._engine.stats["searches"] == n
