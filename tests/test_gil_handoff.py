"""engine._gil_handoff: the switch interval is short only while a search with
queued witness-program compiles is in flight, and restored after the last of
overlapping searches (threads of MultiDevice) ends."""
import sys
import threading

from mythril_amd import engine


def test_interval_short_inside_and_restored():
    before = sys.getswitchinterval()
    with engine._gil_handoff(False):
        assert sys.getswitchinterval() == before
    with engine._gil_handoff(True):
        assert sys.getswitchinterval() == min(before, engine.SEARCH_SWITCH_INTERVAL)
        with engine._gil_handoff(True):
            assert sys.getswitchinterval() == min(before, engine.SEARCH_SWITCH_INTERVAL)
        assert sys.getswitchinterval() == min(before, engine.SEARCH_SWITCH_INTERVAL)
    assert sys.getswitchinterval() == before


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
    assert sys.getswitchinterval() == min(before, engine.SEARCH_SWITCH_INTERVAL)
    leave.set()
    for t in ts:
        t.join()
    assert sys.getswitchinterval() == before
    assert engine._HANDOFF[0] == 0
