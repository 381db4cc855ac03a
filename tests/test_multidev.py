"""Single-process multi-GPU search (mythril_amd/multidev.py)
on N host-emulator devices: the same witnesses (lowest index per program) and
verdicts as one device, in exhaustive and stop-after-hit modes, with the
between-rounds early stop ending the search once every program has a witness."""
import numpy as np
import pytest

from mythril_amd import isa
from mythril_amd.engine import WitnessEngine, prepare
from mythril_amd.ir import Ctx
from mythril_amd.multidev import MultiDevice
from tests.fakedev import FakeDevice
from tests.test_engine_cpu import holds


def _queries():
    c = Ctx()
    x, y, z = c.var("x", 256), c.var("y", 64), c.var("z", 16)
    qs = [
        [c.app("bvult", x, c.const(1 << 250, 256)), c.app("bvugt", y, c.const(1 << 62, 64))],
        [c.app("=", y, c.const(12345, 64))],                                  # no witness in range
        [c.app("=", c.app("bvand", z, c.const(0xFF, 16)), c.const(0x2A, 16))],
        [c.app("bvult", z, c.const(3, 16))],
    ]
    return c, [prepare(q, c, use_pools=False) for q in qs]


class CountingFake(FakeDevice):
    def __init__(self):
        super().__init__(chunk=256)
        self.calls = 0

    def search(self, dps, seed, begin, count, flags=0):
        self.calls += 1
        return super().search(dps, seed, begin, count, flags)


@pytest.mark.parametrize("ndev", [2, 3, 8])
@pytest.mark.parametrize("flags", [0, isa.FLAG_EARLY_EXIT | isa.FLAG_STOP_AFTER_HIT])
def test_multidevice_equals_single_device(ndev, flags):
    c, qs = _queries()
    single = FakeDevice(chunk=256)
    want, _ = single.search([single.load(q.program) for q in qs], 7, 0, 6000, 0)
    devs = [CountingFake() for _ in range(ndev)]
    md = MultiDevice(devs, round_size=200)
    got, st = md.search([md.load(q.program) for q in qs], 7, 0, 6000, flags)
    assert got == want
    assert want[0] is not None and want[1] is None
    if flags:
        assert st["rounds"] >= 1 and all(d.calls <= st["rounds"] for d in devs)
    else:
        assert st["rounds"] == 1   # exhaustive: one round, the range split evenly


def test_early_stop_between_rounds():
    """Every program witnessed early: the later rounds never launch."""
    c = Ctx()
    z = c.var("z", 8)
    q = prepare([c.app("bvult", z, c.const(200, 8))], c, use_pools=False)
    devs = [CountingFake() for _ in range(4)]
    md = MultiDevice(devs, round_size=64)
    (w,), st = md.search([md.load(q.program)], 3, 0, 1 << 16, isa.FLAG_STOP_AFTER_HIT)
    assert w is not None and st["rounds"] == 1
    assert all(d.calls == 1 for d in devs)


def test_eval_generated_concatenates_device_slices():
    c, qs = _queries()
    md = MultiDevice([FakeDevice() for _ in range(3)])
    mp = md.load(qs[0].program)
    v, _ = md.eval_generated(mp, 9, 100, 3000, trace=False)
    ref, _ = FakeDevice().eval_generated(FakeDevice().load(qs[0].program), 9, 100, 3000)
    assert np.array_equal(v, ref)


def test_engine_on_multidevice_materialises_sound_witnesses():
    c, qs = _queries()
    eng = WitnessEngine(dev=MultiDevice([FakeDevice(chunk=512) for _ in range(4)], round_size=512), seed=11,
                        budget=1 << 13)
    ws = eng.search(qs)
    assert ws[0] is not None and holds(qs[0].conjuncts, ws[0])
    assert ws[1] is None
