"""runtime.DeviceProgram's finalizer never calls into the library (VERDICT r5
item 1): a program collected without free() is queued and freed by its
device at the start of the device's next load / search / close, on the
caller's thread.  A recording stand-in for the library; no GPU."""
import gc
import threading

from mythril_amd import runtime


class _Lib:
    def __init__(self):
        self.calls = []

    def mg_prog_free(self, h):
        self.calls.append(("free", h, threading.current_thread().name))
        return 0

    def mg_free(self, h):
        self.calls.append(("ctx_free", h, threading.current_thread().name))
        return 0


def _device(lib):
    d = runtime.Device.__new__(runtime.Device)
    d.lib, d.handle, d.device = lib, 0x1000, 0
    import weakref
    d._live = weakref.WeakSet()
    d._reap_queue = []
    return d


def test_collected_program_is_freed_by_the_next_call_not_the_collector():
    lib = _Lib()
    dev = _device(lib)
    dp = runtime.DeviceProgram(dev, 0x2000, None)
    dev._live.add(dp)

    def drop():          # the last reference dies on another thread (a collection there)
        nonlocal dp
        dp = None
        gc.collect()
    t = threading.Thread(target=drop, name="collector")
    t.start()
    t.join()
    assert lib.calls == [] and dev._reap_queue == [0x2000]
    dev._reap()
    assert lib.calls == [("free", 0x2000, threading.current_thread().name)]
    assert dev._reap_queue == []


def test_close_frees_queued_programs_first():
    lib = _Lib()
    dev = _device(lib)
    dev._reap_queue.extend([0x10, 0x20])
    dev.close()
    assert [c[:2] for c in lib.calls] == [("free", 0x20), ("free", 0x10), ("ctx_free", 0x1000)]
    assert dev.handle is None


def test_explicit_free_is_immediate():
    lib = _Lib()
    dev = _device(lib)
    dp = runtime.DeviceProgram(dev, 0x3000, None)
    dev._live.add(dp)
    dp.free()
    assert lib.calls == [("free", 0x3000, threading.current_thread().name)]
    del dp
    gc.collect()
    assert dev._reap_queue == []
