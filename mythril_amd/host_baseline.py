"""bench.py's fast CPU baseline: the product's own code built for the host
with an OpenMP candidate loop, timed on the same program and candidate
indices the GPU searches.  Preferred: the program's specialised straight-line
code (mythril_amd/jit.py, the source of the benchmarked gfx950 kernel) compiled
for x86 (``<kernel>_host_omp``, cached in build/jit by build()); else the
interpreter and u256 ALU (csrc/mw_interp.h, mw_alu.h, mw_leaf.h;
build/host/libmw_host_emu.so, mwh_count_omp).  SURVEY §8(d): the
reference z3 path is absent here and on the box, so the CPU baseline is "our
C++ OpenMP evaluator on all host cores, labelled build CPU restatement, not
reference".  Measurement only: the product path never loads this library
(mythril_amd/runtime.py has no CPU fallback)."""
from __future__ import annotations

import ctypes
import os
import time
from typing import Optional, Tuple

import numpy as np

from .compiler import Program
from .runtime import make_desc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "build", "host", "libmw_host_emu.so")
_lib = None


def available() -> bool:
    return os.path.exists(LIB)


def lib():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(LIB)
        L.mwh_count_omp.restype = ctypes.c_longlong
        L.mwh_count_omp.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t,
                                    ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int]
        L.mwh_max_threads.restype = ctypes.c_int
        _lib = L
    return _lib


def cpu_model() -> str:
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def count(p: Program, seed: int, begin: int, n: int, verdicts: bool = False,
          nthreads: int = 0) -> Tuple[int, Optional[np.ndarray]]:
    """(satisfied candidates, verdict vector or None) of [begin, begin+n)."""
    d, keep = make_desc(p)
    v = np.zeros(n, dtype=np.uint8) if verdicts else None
    sat = lib().mwh_count_omp(ctypes.byref(d), seed, begin, n, 0, v.ctypes.data if v is not None else None,
                              nthreads)
    if sat < 0:
        raise RuntimeError(f"mwh_count_omp failed ({sat})")
    return int(sat), v


def specialised(p: Program, compile_if_missing: bool = False):
    """The OpenMP host entry of p's specialised code, or None when its build is
    not in the cache (and compile_if_missing is off: it takes minutes)."""
    from . import jit
    if not compile_if_missing and not jit.is_host_cached([p], openmp=True):
        return None
    path, names = jit.compile_host([p], openmp=True)
    L = ctypes.CDLL(str(path))
    f = getattr(L, names[0] + "_host_omp")
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
    return f


def count_specialised(f, p: Program, seed: int, begin: int, n: int) -> Tuple[int, np.ndarray]:
    pool = np.ascontiguousarray(p.pool, dtype=np.uint32)
    v = np.zeros(n, dtype=np.uint32)
    if f(pool.ctypes.data if pool.size else None, seed, begin, n, v.ctypes.data) != 0:
        raise RuntimeError("specialised host entry failed")
    v8 = v.astype(np.uint8)
    return int(v8.sum()), v8


def baseline(p: Program, seed: int, budget_s: float = 10.0, verdicts: bool = False):
    """Candidate indices 0.. in growing batches until budget_s elapses.
    Returns (record, verdict vector or None)."""
    threads = lib().mwh_max_threads()
    f = specialised(p)
    n, sat, t0, dt, batch = 0, 0, time.perf_counter(), 0.0, max(256, threads * 64)
    parts = []
    while dt < budget_s:
        s, v = count_specialised(f, p, seed, n, batch) if f is not None else count(p, seed, n, batch, verdicts)
        sat += s
        if verdicts:
            parts.append(v)
        n += batch
        dt = time.perf_counter() - t0
        if dt < budget_s / 4:
            batch *= 2
    how = ("the benchmarked kernel's own specialised source (mythril_amd/jit.py) compiled for x86, "
           "<kernel>_host_omp, exhaustive" if f is not None else
           "the product's interpreter and u256 ALU built for the host (csrc/mw_host_emu.cpp mwh_count_omp)")
    rec = {"value": n / dt, "unit": "evals/s", "cores": threads, "kind": "port",
           "sample": f"candidate indices 0..{n - 1} of the same program ({n} evals, {dt:.1f} s): {how}, "
                     f"OpenMP x{threads} - build CPU restatement, not reference (no z3 on the box)",
           "satisfied": sat, "cpu_model": cpu_model(), "os_cpu_count": os.cpu_count(),
           "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}
    return rec, (np.concatenate(parts) if parts else None)
