"""The C-ABI's in-flight call record (mythril_amd/csrc/mw_inflight.h, VERDICT
r5 item 1): a call stuck in a step is named by a watchdog on another thread
(mg_debug_inflight), a slow step names itself on stderr when it ends, and
the library exports the report.  Host-only (tests/native/inflight_check.cpp
under ThreadSanitizer)."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
SRC = ROOT / "tests" / "native" / "inflight_check.cpp"


def test_stuck_call_is_reported_and_slow_steps_name_themselves(tmp_path):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    exe = tmp_path / "ic"
    r = subprocess.run([gxx, "-std=c++17", "-O1", "-g", "-fsanitize=thread", "-pthread", str(SRC), "-o", str(exe)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120,
                       env={"MYTHRIL_AMD_SLOW_STEP_MS": "50", "TSAN_OPTIONS": "halt_on_error=1"})
    assert r.returncode == 0 and r.stdout.rstrip().endswith("OK"), (r.stdout, r.stderr[-3000:])
    assert "mg_test_call/blocked arg=4096" in r.stdout
    # the blocked step ran past 50 ms: named on stderr when it ended
    assert "[mythril_amd] slow step: mg_test_call/blocked (4096)" in r.stderr
    assert "WARNING: ThreadSanitizer" not in r.stderr


def test_library_exports_the_report():
    from mythril_amd import runtime
    if not os.path.exists(runtime.LIB_PATH):
        pytest.skip("library not built")
    lib = runtime.load_library()
    assert lib.mg_debug_inflight(None, 0) == 0      # no call in flight here
    assert runtime.inflight() == ""


def test_every_device_call_is_marked():
    src = (ROOT / "mythril_amd" / "csrc" / "mw_kernels.hip").read_text()
    for fn in ("mg_init", "mg_free", "mg_prog_load", "mg_prog_free", "mg_search", "mg_eval", "mg_eval_generated",
               "mg_witness_leaves", "mg_eval_program", "mg_prog_attach_kernel", "mg_prog_attach_asm", "mg_keccak256",
               "mg_keccak256_device"):
        body = src[src.index(f"int {fn}("):]
        body = body[:body.index("\n}\n")]
        assert f'mw::CallMark mark("{fn}")' in body, fn
