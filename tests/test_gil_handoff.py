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
