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
