"""The C-ABI's handle lifetimes (mythril_amd/csrc/mw_handles.h, used by
mw_kernels.hip for every entry point) under ThreadSanitizer and
AddressSanitizer: tests/native/handles_stress.cpp frees contexts while other
threads load, search and free their programs.
Host-only: the protocol has no device code."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
SRC = ROOT / "tests" / "native" / "handles_stress.cpp"


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_handle_protocol_under_sanitizer(tmp_path, san):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    exe = tmp_path / "hs"
    r = subprocess.run([gxx, "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-sanitize-recover=all",
                        "-pthread", str(SRC), "-o", str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([str(exe), "150"], capture_output=True, text=True, timeout=240,
                       env={"TSAN_OPTIONS": "halt_on_error=1", "ASAN_OPTIONS": "detect_leaks=1"})
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert r.stdout.startswith("OK") and "WARNING" not in r.stderr


def test_product_library_uses_the_registry():
    """Every entry point of mw_kernels.hip resolves handles through the
    registry: no raw handle dereference remains."""
    src = (ROOT / "mythril_amd" / "csrc" / "mw_kernels.hip").read_text()
    assert "mw::Registry<Ctx, Prog> g_reg" in src
    for fn in ("mg_free", "mg_prog_free", "mg_search", "mg_eval", "mg_eval_generated", "mg_prog_attach_kernel",
               "mg_prog_attach_asm", "mg_prog_engine", "mg_valu_peak", "mg_keccak256_device"):
        body = src[src.index(f"int {fn}("):]
        body = body[:body.index("\n}\n")]
        assert "g_reg" in body, fn
