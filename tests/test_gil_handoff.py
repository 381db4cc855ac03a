"""engine._gil_handoff: the switch interval is short only while a search with
queued witness-program compiles is in flight, and restored after the last of
overlapping searches (threads of MultiDevice) ends."""
import math
import sys
import threading

from mythril_amd import engine


def _short(before):
    """the interval inside a handoff (the interpreter stores it in microseconds)"""
    return math.isclose(sys.getswitchinterval(), min(before, engine.SEARCH_SWITCH_INTERVAL), rel_tol=1e-6)


def _is(x):
    return math.isclose(sys.getswitchinterval(), x, rel_tol=1e-6)


def test_interval_short_inside_and_restored():
    before = sys.getswitchinterval()
    with engine._gil_handoff(False):
        assert _is(before)
    with engine._gil_handoff(True):
        assert _short(before)
        with engine._gil_handoff(True):
            assert _short(before)
        assert _short(before)
    assert _is(before)


def test_overlapping_threads_restore_once():
    before = sys.getswitchinterval()
    inside = threading.Barrier(4)
    leave = threading.Event()

    def run():
        with engine._gil_handoff(True):
            inside.wait()
            leave.wait(5)
    ts = [threading.Thread(target=run) for _ in range(3)]
    for t in ts:
        t.start()
    inside.wait()
    assert _short(before)
    leave.set()
    for t in ts:
        t.join()
    assert _is(before)
    assert engine._HANDOFF[0] == 0


def test_a_change_made_meanwhile_is_kept():
    """the saved interval is put back only if the interval is still
    the one the hand-off set; another component's change stays."""
    before = sys.getswitchinterval()
    try:
        with engine._gil_handoff(True):
            sys.setswitchinterval(0.002)
        assert _is(0.002)
    finally:
        sys.setswitchinterval(before)


def test_search_withdraws_queued_compiles_of_misses(monkeypatch):
    """a search that finds nothing leaves no witness-program
    compile queued on the host thread (nor when the device raises).  The
    thread is off by default since round 6 (MYTHRIL_AMD_WITNESS_THREAD=1)."""
    monkeypatch.setattr(engine, "WITNESS_THREAD", True)
    from mythril_amd.engine import WitnessEngine, prepare
    from mythril_amd.ir import Ctx
    from tests.fakedev import FakeDevice
    c = Ctx()
    arr = c.array("cd", 256, 8)
    x = c.var("x", 256)
    # a cell with a variable index: the witness program is queued for compile
    miss = [c.app("=", c.app("select", arr, x), c.const(7, 8)), c.app("=", x, c.const(3, 256)),
            c.app("=", x, c.const(4, 256))]
    eng = WitnessEngine(dev=FakeDevice(chunk=256), budget=1 << 10)
    q = prepare(miss, c)
    assert eng.search([q]) == [None]
    assert q._trace_future is None

    class Boom(FakeDevice):
        def search(self, *a, **k):
            raise RuntimeError("device")
    q2 = prepare(miss, c)
    eng2 = WitnessEngine(dev=Boom(chunk=256), budget=1 << 10)
    try:
        eng2.search([q2])
    except RuntimeError:
        pass
    assert q2._trace_future is None
