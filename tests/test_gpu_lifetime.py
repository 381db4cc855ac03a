"""C-ABI handle lifetimes on the device.  Round 2's sticky
"invalid device ordinal" was a program freed after its context; the library
now keeps a registry of live handles, so the reversed order is an MG_E_ARG
from any binder, and the device stays usable."""
import pytest

from mythril_amd.compiler import compile_program
from mythril_amd.ir import Ctx

pytestmark = pytest.mark.gpu


def _prog():
    c = Ctx()
    x = c.var("x", 256)
    return compile_program([c.app("bvult", x, c.const(1 << 255, 256))])


def test_program_freed_after_its_context():
    from mythril_amd.runtime import Device
    dev = Device(0)
    lib = dev.lib
    dp = dev.load(_prog())
    h_prog, h_ctx = dp.handle, dev.handle
    # free the context first through the raw C-ABI (what another binder could do)
    assert lib.mg_free(h_ctx) == 0            # frees the still-loaded program with it
    dev.handle = None
    assert lib.mg_prog_free(h_prog) == -1     # no use-after-free: rejected
    assert b"not a live program" in lib.mg_last_error()
    assert lib.mg_free(h_ctx) == -1           # double free of the context: rejected
    dp.handle = None
    # the device is still usable: a new context searches correctly
    dev2 = Device(0)
    try:
        dp2 = dev2.load(_prog())
        (found,), st = dev2.search([dp2], 1, 0, 1 << 12, 0)
        assert found is not None and found < 8 and st["evals"] == 1 << 12
        h2 = dp2.handle
        dp2.free()
        assert lib.mg_prog_free(h2) == -1     # double free of a program: rejected
        out = (__import__("ctypes").c_uint64 * 1)()
        arr = (__import__("ctypes").c_void_p * 1)(h2)
        assert lib.mg_search(dev2.handle, arr, 1, 1, 0, 256, 0, out, None) == -1
    finally:
        dev2.close()


def test_close_frees_loaded_programs():
    from mythril_amd.runtime import Device
    dev = Device(0)
    dps = [dev.load(_prog()) for _ in range(4)]
    handles = [dp.handle for dp in dps]
    lib = dev.lib
    assert lib.mg_free(dev.handle) == 0
    dev.handle = None
    for h, dp in zip(handles, dps):
        assert lib.mg_prog_free(h) == -1
        dp.handle = None


def test_stale_handle_refused_after_a_new_load():
    """Handles are ids that are never reused: a freed program's
    handle stays refused after later loads, which may get its memory."""
    import ctypes

    from mythril_amd.runtime import Device
    dev = Device(0)
    try:
        lib = dev.lib
        dp = dev.load(_prog())
        old = dp.handle
        dp.free()
        fresh = [dev.load(_prog()) for _ in range(8)]
        assert old not in [d.handle for d in fresh]
        assert lib.mg_prog_free(old) == -1
        out = (ctypes.c_uint64 * 1)()
        assert lib.mg_search(dev.handle, (ctypes.c_void_p * 1)(old), 1, 1, 0, 256, 0, out, None) == -1
        (found,), _ = dev.search([fresh[0]], 1, 0, 1 << 12, 0)
        assert found is not None
        for d in fresh:
            d.free()
    finally:
        dev.close()


def test_context_freed_while_other_threads_search():
    """mg_free waits for the call in flight on another thread and frees the
    programs with the context; later calls with those handles are refused."""
    import ctypes
    import threading

    from mythril_amd.runtime import Device
    dev = Device(0)
    lib = dev.lib
    dps = [dev.load(_prog()) for _ in range(4)]
    ctx = dev.handle
    handles = [dp.handle for dp in dps]
    rcs = []

    def searcher(h):
        out = (ctypes.c_uint64 * 1)()
        for _ in range(20):
            rcs.append(lib.mg_search(ctx, (ctypes.c_void_p * 1)(h), 1, 1, 0, 1 << 16, 0, out, None))

    ts = [threading.Thread(target=searcher, args=(h,)) for h in handles]
    for t in ts:
        t.start()
    assert lib.mg_free(ctx) == 0
    for t in ts:
        t.join()
    dev.handle = None
    for dp in dps:
        dp.handle = None
    assert rcs and set(rcs) <= {0, -1}
    for h in handles:
        assert lib.mg_prog_free(h) == -1
    dev2 = Device(0)                      # the device is still usable
    try:
        dp2 = dev2.load(_prog())
        (found,), _ = dev2.search([dp2], 1, 0, 1 << 12, 0)
        assert found is not None
        dp2.free()
    finally:
        dev2.close()
