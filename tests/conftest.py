import faulthandler
import os
import sys
import threading
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# GPU tests report a stall themselves (a GPU run went
# silent inside one test and the box's silence watchdog, 3 minutes, killed
# it before pytest-timeout's 300 s could dump anything).  Every GPU test:
# * gets a pytest-timeout of GPU_TEST_TIMEOUT s (thread method: dumps every
#   thread's stack, then ends the run), below the box's 180 s silence limit;
# * after GPU_WATCHDOG_S s, and every 30 s after, prints on stderr which test
#   is running, the C-ABI calls in flight with the step each is in
#   (runtime.inflight(): mg_debug_inflight, lock-free) and every thread's
#   Python stack (faulthandler).
GPU_TEST_TIMEOUT = int(os.environ.get("MW_GPU_TEST_TIMEOUT", "150"))
GPU_WATCHDOG_S = float(os.environ.get("MW_GPU_WATCHDOG_S", "60"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pytest_collection_modifyitems(config, items):
    if not config.pluginmanager.hasplugin("timeout"):
        return
    for item in items:
        if item.get_closest_marker("gpu") is not None and item.get_closest_marker("timeout") is None:
            item.add_marker(pytest.mark.timeout(GPU_TEST_TIMEOUT, method="thread"))


def _stall_report(nodeid: str, t0: float) -> None:
    err = sys.__stderr__
    try:
        from mythril_amd import runtime
        calls = runtime.inflight()
    except Exception as e:   # noqa: BLE001 - a report, never a failure
        calls = f"(no report: {e})\n"
    calls = calls or "(none)\n"
    err.write(f"\n[watchdog {time.strftime('%H:%M:%S')}] {nodeid} running for {time.monotonic() - t0:.0f} s; "
              f"C-ABI calls in flight:\n{calls}")
    err.flush()
    faulthandler.dump_traceback(file=err, all_threads=True)
    err.flush()


@pytest.hookimpl(hookwrapper=True)
def pytest_runtest_protocol(item, nextitem):
    if item.get_closest_marker("gpu") is None or GPU_WATCHDOG_S <= 0:
        yield
        return
    done = threading.Event()
    t0 = time.monotonic()

    def watch():
        wait = GPU_WATCHDOG_S
        while not done.wait(wait):
            _stall_report(item.nodeid, t0)
            wait = 30.0
    th = threading.Thread(target=watch, name="mw-test-watchdog", daemon=True)
    th.start()
    try:
        yield
    finally:
        done.set()
        th.join(timeout=5)
