"""ctypes binding of the host build of the interpreter (build/host/libmw_host_emu.so).

``csrc/mw_host_emu.cpp`` compiles the very interpreter, ALU and candidate
generator the gfx950 kernels run (mw_interp.h, mw_alu.h, mw_leaf.h) for x86.
It is never a fallback for the device path (runtime.py has none).  Its uses:
tests, and build-time workload preparation — e.g. planting the C5 witness on
the CPU so that ``__graft_entry__.build()`` can pre-compile the benchmark's
specialised kernel (mythril_amd/jit.py) into the in-tree cache, bit for bit
the program bench.py later builds on the device.
"""
from __future__ import annotations

import ctypes
import os
from typing import Callable, List, Sequence

import numpy as np

from .compiler import Program, compile_program
from .runtime import MgProgDesc, make_desc, unpack_trace

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST_EMU = os.path.join(ROOT, "build", "host", "libmw_host_emu.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(HOST_EMU):
            from .build import build_host_emu
            build_host_emu()
        L = ctypes.CDLL(HOST_EMU)
        L.mwh_eval.restype = ctypes.c_int
        L.mwh_eval.argtypes = [ctypes.POINTER(MgProgDesc), ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                               ctypes.c_size_t, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
        L.mwh_div_counts.restype = ctypes.c_int
        L.mwh_div_counts.argtypes = [ctypes.POINTER(MgProgDesc), ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t,
                                     ctypes.c_void_p]
        L.mg_last_error.restype = ctypes.c_char_p
        _lib = L
    return _lib


def eval_generated(p: Program, seed: int, begin: int, n: int):
    """Verdicts and trace rows of generated candidates [begin, begin+n) (host build)."""
    d, keep = make_desc(p)
    v = np.zeros(n, dtype=np.uint32)
    t = np.zeros(max(p.n_trace_rows, 1) * n, dtype=np.uint32)
    rc = lib().mwh_eval(ctypes.byref(d), None, seed, begin, n, 0, v.ctypes.data, t.ctypes.data)
    if rc != 0:
        raise RuntimeError(lib().mg_last_error().decode())
    return v, t.reshape(max(p.n_trace_rows, 1), n)


def div_counts(p: Program, seed: int, begin: int, n: int) -> dict:
    """Division path counts (mg_stats.lane_div_* names) of the host build over
    generated candidates [begin, begin+n); a host 'wave' is one candidate."""
    d, keep = make_desc(p)
    out = np.zeros(4, dtype=np.uint64)
    rc = lib().mwh_div_counts(ctypes.byref(d), seed, begin, n, out.ctypes.data)
    if rc != 0:
        raise RuntimeError(lib().mg_last_error().decode())
    return {"lane_div_steps": int(out[0]), "lane_div_full": int(out[1]), "lane_div_short": int(out[2]),
            "lane_div_general": int(out[3])}


def term_values(terms: Sequence, index: int, seed: int) -> List[int]:
    """Values of `terms` at generated candidate `index` (synth.build_c5's evaluate)."""
    p = compile_program([], trace=list(terms))
    _, tr = eval_generated(p, seed, index, 1)
    return [unpack_trace(p, tr, t)[0] for t in terms]
