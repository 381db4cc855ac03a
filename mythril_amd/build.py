"""Build the native libraries in-tree (hipcc cross-compiles gfx950 without a GPU).

  mythril_amd/lib/libmythril_witness.so   product: gfx950 kernels + C-ABI + the host compiler
  build/host/libmw_host_emu.so            test-only CPU build of the same interpreter
  oracle/build/liboracle.so               test-only C restatement (built by oracle/Makefile)
  mythril_amd/lib/asmjit_template.s       the assembled kernels' template (gfx950 assembly,
                                          mythril_amd/asmjit.py fills in a program's body)

Usage: python -m mythril_amd.build [--force]
"""
from __future__ import annotations

import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "mythril_amd" / "csrc"
LIB = ROOT / "mythril_amd" / "lib" / "libmythril_witness.so"
HOST_EMU = ROOT / "build" / "host" / "libmw_host_emu.so"
ARCH = os.environ.get("MW_OFFLOAD_ARCH", "gfx950")

DEVICE_SRCS = ["mw_kernels.hip", "mw_validate.cpp", "mw_compile.cpp"]
HOST_SRCS = ["mw_host_emu.cpp", "mw_validate.cpp"]
HEADERS = ["mw_isa.h", "mw_prog.h", "mw_alu.h", "mw_interp.h", "mw_leaf.h", "mw_keccak.h", "mw_asm_interp.inc",
           "mw_asm_abi.h", "mw_handles.h"]
ASMJIT_TEMPLATE = ROOT / "mythril_amd" / "lib" / "asmjit_template.s"   # package data


def _hipcc() -> str:
    for c in ("/opt/rocm/bin/hipcc", "hipcc"):
        if os.path.exists(c) or c == "hipcc":
            return c
    return "hipcc"


def _stale(target: Path, srcs) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    deps = [CSRC / s for s in srcs] + [CSRC / h for h in HEADERS] + [ROOT / "include" / h for h in
                                                                     ("mythril_witness.h", "mythril_compile.h")]
    return any(d.stat().st_mtime > t for d in deps if d.exists())


def _run(cmd):
    print("+", " ".join(str(c) for c in cmd), flush=True)
    subprocess.run([str(c) for c in cmd], check=True, cwd=CSRC)


def build_device(force: bool = False) -> Path:
    if force or _stale(LIB, DEVICE_SRCS):
        LIB.parent.mkdir(parents=True, exist_ok=True)
        tmp = LIB.with_suffix(".so.tmp")
        _run([_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
              # -Wno-inline-asm: the asm interpreter clobbers m0 (s_set_gpr_idx_on) on purpose
              "-Wno-unused-result", "-Wno-unused-value", "-Wno-inline-asm", *DEVICE_SRCS, "-o", tmp])
        os.replace(tmp, LIB)
    return LIB


def build_host_emu(force: bool = False) -> Path:
    if force or _stale(HOST_EMU, HOST_SRCS):
        HOST_EMU.parent.mkdir(parents=True, exist_ok=True)
        tmp = HOST_EMU.with_suffix(".so.tmp")
        # host-only compile of the same headers (no device code in these TUs)
        # OpenMP: mwh_count_omp, bench.py's CPU baseline on the product's ALU
        _run([_hipcc(), "-O2", "-std=c++17", "-fPIC", "-shared", "-D__HIP_PLATFORM_AMD__", "-fopenmp",
              *HOST_SRCS, "-o", tmp, "-Wl,-rpath,/opt/rocm/llvm/lib"])
        os.replace(tmp, HOST_EMU)
    return HOST_EMU


def build_asmjit_template(force: bool = False) -> Path:
    """hipcc compiles the assembled kernels' shell to gfx950 assembly once; the
    runtime only assembles (mythril_amd/asmjit.py)."""
    if force or _stale(ASMJIT_TEMPLATE, ["mw_asmjit_shell.hip"]):
        ASMJIT_TEMPLATE.parent.mkdir(parents=True, exist_ok=True)
        tmp = ASMJIT_TEMPLATE.with_suffix(".s.tmp")
        _run([_hipcc(), f"--offload-arch={ARCH}", "--cuda-device-only", "-S", "-O3", "-std=c++17",
              "-Wno-inline-asm", "-Wno-unused-command-line-argument", "mw_asmjit_shell.hip", "-o", tmp])
        os.replace(tmp, ASMJIT_TEMPLATE)
    return ASMJIT_TEMPLATE


def build_oracle(force: bool = False) -> None:
    mk = ROOT / "oracle" / "Makefile"
    if mk.exists():
        subprocess.run(["make", "-C", str(mk.parent)] + (["-B"] if force else []), check=True)


def build_all(force: bool = False) -> None:
    build_device(force)
    build_asmjit_template(force)
    build_host_emu(force)
    build_oracle(force)


if __name__ == "__main__":
    build_all("--force" in sys.argv)
