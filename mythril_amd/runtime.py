"""ctypes binding of ``libmythril_witness.so`` (include/mythril_witness.h).

This is the only way the product reaches the device.  There is no CPU
fallback: if the library or a GPU is missing, :func:`load_library` /
:class:`Device` raise :class:`EngineUnavailable`, and callers (the drop-in
``get_model``) route the query to z3 exactly as the reference does.  ctypes
releases the GIL for the duration of each call, like z3's own bindings.
"""
from __future__ import annotations

import ctypes
import os
import threading
import weakref
from typing import List, Optional, Sequence, Tuple

import numpy as np

from .compiler import Program

# MYTHRIL_AMD_LIB: load another build of the library (A/B measurements)
LIB_PATH = os.environ.get("MYTHRIL_AMD_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib",
                                                             "libmythril_witness.so")
MG_NONE = (1 << 64) - 1


class EngineUnavailable(RuntimeError):
    """The HIP extension or the device is not available."""


class EngineError(RuntimeError):
    pass


class MgProgDesc(ctypes.Structure):
    _fields_ = [
        ("code", ctypes.c_void_p), ("ncode_words", ctypes.c_size_t),
        ("consts", ctypes.c_void_p), ("nconst_words", ctypes.c_size_t),
        ("leaves", ctypes.c_void_p), ("nleaves", ctypes.c_size_t),
        ("pool", ctypes.c_void_p), ("npool_words", ctypes.c_size_t),
        ("n_spill", ctypes.c_uint32), ("n_trace_rows", ctypes.c_uint32),
        ("n_input_rows", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
        ("ops_per_eval", ctypes.c_uint64),
    ]


class MgStats(ctypes.Structure):
    _fields_ = [("kernel_ms", ctypes.c_double), ("wall_ms", ctypes.c_double),
                ("evals", ctypes.c_uint64), ("launches", ctypes.c_uint64), ("ops", ctypes.c_double),
                ("lane_div_steps", ctypes.c_uint64), ("lane_div_full", ctypes.c_uint64),
                ("lane_div_short", ctypes.c_uint64), ("lane_div_general", ctypes.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_P = ctypes.c_void_p
_lib = None
_lib_lock = threading.Lock()

SIGNATURES = {
    "mg_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "mg_init": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(_P)]),
    "mg_free": (ctypes.c_int, [_P]),
    "mg_prog_load": (ctypes.c_int, [_P, ctypes.POINTER(MgProgDesc), ctypes.POINTER(_P)]),
    "mg_prog_free": (ctypes.c_int, [_P]),
    "mg_prog_attach_kernel": (ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]),
    "mg_prog_attach_asm": (ctypes.c_int, [_P, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p]),
    "mg_prog_has_kernel": (ctypes.c_int, [_P]),
    "mg_prog_engine": (ctypes.c_int, [_P]),
    "mg_search": (ctypes.c_int, [_P, ctypes.POINTER(_P), ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64,
                                 ctypes.c_uint64, ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64),
                                 ctypes.POINTER(MgStats)]),
    "mg_search_begin": (ctypes.c_int, [_P, ctypes.POINTER(_P), ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64,
                                       ctypes.c_uint64, ctypes.c_uint32]),
    "mg_search_end": (ctypes.c_int, [_P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(MgStats),
                                     ctypes.POINTER(ctypes.POINTER(MgProgDesc)), ctypes.POINTER(_P),
                                     ctypes.POINTER(ctypes.c_int32)]),
    "mg_eval": (ctypes.c_int, [_P, _P, _P, ctypes.c_size_t, _P, _P]),
    "mg_eval_generated": (ctypes.c_int, [_P, _P, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_size_t, _P, _P]),
    "mg_witness_leaves": (ctypes.c_int, [_P, _P, ctypes.c_uint64, ctypes.c_uint64, _P]),
    "mg_eval_program": (ctypes.c_int, [_P, ctypes.POINTER(MgProgDesc), ctypes.c_uint64, ctypes.c_uint64,
                                       ctypes.c_size_t, _P, _P]),
    "mg_keccak256": (ctypes.c_int, [_P, _P, ctypes.c_size_t, _P, _P, ctypes.c_size_t, _P, ctypes.POINTER(MgStats)]),
    "mg_keccak256_device": (ctypes.c_int, [_P, _P, _P, _P, ctypes.c_size_t, _P, ctypes.POINTER(MgStats)]),
    "mg_validate_desc": (ctypes.c_int, [ctypes.POINTER(MgProgDesc)]),
    "mg_valu_peak": (ctypes.c_int, [_P, ctypes.c_uint32, ctypes.POINTER(ctypes.c_double),
                                    ctypes.POINTER(ctypes.c_double)]),
    "mg_last_error": (ctypes.c_char_p, []),
    "mg_debug_inflight": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t]),
    "mg_debug_step_times": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t]),
}


def bind(lib):
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    return lib


def load_library(path: str = LIB_PATH):
    """Load the HIP library; raises EngineUnavailable (never falls back)."""
    global _lib
    with _lib_lock:
        if _lib is None:
            if not os.path.exists(path):
                raise EngineUnavailable(f"HIP extension not built: {path} (run python -m mythril_amd.build)")
            try:
                _lib = bind(ctypes.CDLL(path))
            except OSError as e:
                raise EngineUnavailable(f"cannot load {path}: {e}") from e
        return _lib


def _ptr(a: np.ndarray) -> Optional[int]:
    return a.ctypes.data if a is not None and a.size else None


def make_desc(p: Program) -> Tuple[MgProgDesc, list]:
    keep = [np.ascontiguousarray(x, dtype=np.uint32) for x in (p.code, p.consts, p.leaves, p.pool)]
    code, consts, leaves, pool = keep
    d = MgProgDesc(
        code=_ptr(code), ncode_words=code.size,
        consts=_ptr(consts), nconst_words=consts.size,
        leaves=_ptr(leaves), nleaves=leaves.size // 8,
        pool=_ptr(pool), npool_words=pool.size,
        n_spill=p.n_spill, n_trace_rows=p.n_trace_rows, n_input_rows=p.n_input_rows, reserved=0,
        ops_per_eval=p.ops_per_eval)
    return d, keep


def _check(lib, rc: int, what: str):
    if rc != 0:
        msg = lib.mg_last_error()
        raise EngineError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


class DeviceProgram:
    def __init__(self, dev: "Device", handle: int, prog: Program):
        self.dev = dev
        self.handle = handle
        self.prog = prog
        self.kernel: Optional[str] = None   # specialised kernel name, if attached
        self.assembled: Optional[str] = None  # assembled kernel name (mythril_amd.asmjit), if attached

    def free(self):
        # a program never outlives its context: Device.close() frees the
        # programs still loaded, and a freed context is never touched again
        if self.handle and self.dev.handle:
            self.dev.lib.mg_prog_free(self.handle)
            self.dev._live.discard(self)
        self.handle = None

    def __del__(self):  # pragma: no cover - best effort
        # A finalizer runs on whichever thread the garbage collector happens
        # to run (the witness-program thread, in the middle of another call's
        # Python wrapper): it only queues the handle, and the device frees it
        # at the start of its next call from its own caller (Device._reap),
        # so no library call (mg_prog_free: a module unload, hipFree) ever
        # runs from a collection.
        try:
            if self.handle and self.dev.handle:
                self.dev._reap_queue.append(self.handle)
            self.handle = None
        except Exception:
            pass


class Device:
    """One HIP device context (one process per GPU; see mythril_amd.distributed)."""

    def __init__(self, device: int = 0):
        self.lib = load_library()
        n = ctypes.c_int(0)
        rc = self.lib.mg_device_count(ctypes.byref(n))
        if rc != 0 or n.value == 0:
            raise EngineUnavailable("no HIP device visible")
        h = _P()
        _check(self.lib, self.lib.mg_init(device, ctypes.byref(h)), "mg_init")
        self.handle = h.value
        self.device = device
        self._live = weakref.WeakSet()   # programs loaded and not yet freed
        self._reap_queue: List[int] = []    # handles of programs collected without free() (DeviceProgram.__del__)

    def _reap(self):
        """Free the programs the garbage collector queued (list.pop is atomic)."""
        q = self._reap_queue
        while q:
            try:
                h = q.pop()
            except IndexError:
                break
            if self.handle:
                self.lib.mg_prog_free(h)

    def close(self):
        if self.handle:
            self._reap()
            for dp in list(self._live):
                dp.free()
            self.lib.mg_free(self.handle)
            self.handle = None

    def load(self, p: Program) -> DeviceProgram:
        if not self.handle:
            raise EngineError("device context is closed")
        if self._reap_queue:
            self._reap()
        d, keep = make_desc(p)
        h = _P()
        _check(self.lib, self.lib.mg_prog_load(self.handle, ctypes.byref(d), ctypes.byref(h)), "mg_prog_load")
        dp = DeviceProgram(self, h.value, p)
        self._live.add(dp)
        return dp

    def attach_kernel(self, dp: DeviceProgram, image: bytes, name: str) -> None:
        """Bind a specialised code object (mythril_amd.jit) to a loaded program."""
        _check(self.lib, self.lib.mg_prog_attach_kernel(dp.handle, image, len(image), name.encode()),
               "mg_prog_attach_kernel")
        dp.kernel = name

    def attach_asm(self, dp: DeviceProgram, image: bytes, name: str) -> None:
        """Bind an assembled code object (mythril_amd.asmjit) to a loaded program."""
        _check(self.lib, self.lib.mg_prog_attach_asm(dp.handle, image, len(image), name.encode()),
               "mg_prog_attach_asm")
        dp.assembled = name

    def has_kernel(self, dp: DeviceProgram) -> bool:
        return bool(self.lib.mg_prog_has_kernel(dp.handle))

    ENGINES = ("interp", "asm", "jit", "asmjit")

    def engine_of(self, dp: DeviceProgram) -> str:
        """Which kernel searches this program (mg_prog_engine)."""
        rc = self.lib.mg_prog_engine(dp.handle)
        if rc < 0:
            _check(self.lib, rc, "mg_prog_engine")
        return self.ENGINES[rc]

    def search(self, progs: Sequence[DeviceProgram], seed: int, begin: int, count: int,
               flags: int = 0) -> Tuple[List[Optional[int]], dict]:
        if self._reap_queue:
            self._reap()
        arr = (_P * len(progs))(*[dp.handle for dp in progs])
        out = (ctypes.c_uint64 * len(progs))()
        st = MgStats()
        _check(self.lib, self.lib.mg_search(self.handle, arr, len(progs), seed & ((1 << 64) - 1), begin, count,
                                            flags, out, ctypes.byref(st)), "mg_search")
        res = [None if v == MG_NONE else int(v) for v in out]
        return res, st.as_dict()

    def search_begin(self, progs: Sequence[DeviceProgram], seed: int, begin: int, count: int,
                     flags: int = 0) -> None:
        """mg_search_begin: enqueue a search and return at once; search_end
        completes it (the caller may compile witness programs meanwhile)."""
        if self._reap_queue:
            self._reap()
        arr = (_P * len(progs))(*[dp.handle for dp in progs])
        _check(self.lib, self.lib.mg_search_begin(self.handle, arr, len(progs), seed & ((1 << 64) - 1), begin, count,
                                                  flags), "mg_search_begin")
        self._begun = len(progs)

    def search_end(self, witness: Optional[Sequence[Optional[Program]]] = None):
        """mg_search_end: (lowest satisfying index per program or None, stats,
        traces): traces[i] is the trace rows of witness[i] evaluated at
        program i's index (one column, as eval_generated(..., count=1)
        returns it), or None (no witness program, no hit, or not on the asm
        interpreter: the caller evaluates it)."""
        n = getattr(self, "_begun", 0)
        self._begun = 0
        out = (ctypes.c_uint64 * max(1, n))()
        st = MgStats()
        traces = [None] * n
        if witness is not None:
            descs = (ctypes.POINTER(MgProgDesc) * n)()
            bufs = (_P * n)()
            traced = (ctypes.c_int32 * n)()
            keep, arrays = [], [None] * n
            for i, p in enumerate(witness):
                if p is None or not p.n_trace_rows:
                    continue
                d, k = make_desc(p)
                keep.append((d, k))
                descs[i] = ctypes.pointer(d)
                arrays[i] = np.zeros(p.n_trace_rows, dtype=np.uint32)
                bufs[i] = arrays[i].ctypes.data
            _check(self.lib, self.lib.mg_search_end(self.handle, out, ctypes.byref(st), descs, bufs, traced),
                   "mg_search_end")
            traces = [arrays[i].reshape(-1, 1) if traced[i] else None for i in range(n)]
        else:
            _check(self.lib, self.lib.mg_search_end(self.handle, out, ctypes.byref(st), None, None, None),
                   "mg_search_end")
        return [None if out[i] == MG_NONE else int(out[i]) for i in range(n)], st.as_dict(), traces

    def eval(self, dp: DeviceProgram, leaves_soa: Optional[np.ndarray], ncand: int,
             trace: bool = True) -> Tuple[np.ndarray, Optional[np.ndarray]]:
        v = np.zeros(ncand, dtype=np.uint32)
        t = np.zeros(dp.prog.n_trace_rows * ncand, dtype=np.uint32) if trace and dp.prog.n_trace_rows else None
        inp = np.ascontiguousarray(leaves_soa, dtype=np.uint32) if leaves_soa is not None else None
        _check(self.lib, self.lib.mg_eval(self.handle, dp.handle, _ptr(inp) if inp is not None else None, ncand,
                                          v.ctypes.data, _ptr(t) if t is not None else None), "mg_eval")
        return v, (t.reshape(dp.prog.n_trace_rows, ncand) if t is not None else None)

    def eval_generated(self, dp: DeviceProgram, seed: int, begin: int, count: int,
                       trace: bool = True) -> Tuple[np.ndarray, Optional[np.ndarray]]:
        v = np.zeros(count, dtype=np.uint32)
        t = np.zeros(dp.prog.n_trace_rows * count, dtype=np.uint32) if trace and dp.prog.n_trace_rows else None
        _check(self.lib, self.lib.mg_eval_generated(self.handle, dp.handle, seed & ((1 << 64) - 1), begin, count,
                                                    v.ctypes.data, _ptr(t) if t is not None else None),
               "mg_eval_generated")
        return v, (t.reshape(dp.prog.n_trace_rows, count) if t is not None else None)

    def eval_program(self, p: Program, seed: int, begin: int, count: int = 1,
                     trace: bool = True) -> Tuple[np.ndarray, Optional[np.ndarray]]:
        """load + eval_generated + free of a program that is not kept, in one
        library call (mg_eval_program)."""
        if not self.handle:
            raise EngineError("device context is closed")
        d, keep = make_desc(p)
        v = np.zeros(count, dtype=np.uint32)
        t = np.zeros(p.n_trace_rows * count, dtype=np.uint32) if trace and p.n_trace_rows else None
        _check(self.lib, self.lib.mg_eval_program(self.handle, ctypes.byref(d), seed & ((1 << 64) - 1), begin, count,
                                                  v.ctypes.data, _ptr(t) if t is not None else None),
               "mg_eval_program")
        return v, (t.reshape(p.n_trace_rows, count) if t is not None else None)

    def witness_leaves(self, dp: DeviceProgram, seed: int, index: int) -> List[int]:
        """The value of every leaf of dp's program at candidate index, in
        leaf-table order (mg_witness_leaves), masked to the leaf's width."""
        p = dp.prog
        n = len(p.leaf_nodes)
        out = np.zeros(max(1, n) * 8, dtype=np.uint32)
        _check(self.lib, self.lib.mg_witness_leaves(self.handle, dp.handle, seed & ((1 << 64) - 1), index,
                                                    out.ctypes.data), "mg_witness_leaves")
        vals = []
        for i, node in enumerate(p.leaf_nodes):
            v = 0
            for k in range(8):
                v |= int(out[8 * i + k]) << (32 * k)
            w = 1 if node.width == 0 else node.width
            vals.append(v & ((1 << w) - 1))
        return vals

    def keccak256(self, msgs: Sequence[bytes]) -> Tuple[List[bytes], dict]:
        n = len(msgs)
        if n == 0:
            return [], {}
        data = np.frombuffer(b"".join(msgs) or b"\0", dtype=np.uint8)
        lens = np.array([len(m) for m in msgs], dtype=np.uint32)
        offs = np.zeros(n, dtype=np.uint64)
        if n > 1:
            offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
        out = np.zeros(32 * n, dtype=np.uint8)
        st = MgStats()
        _check(self.lib, self.lib.mg_keccak256(self.handle, data.ctypes.data, sum(len(m) for m in msgs),
                                               offs.ctypes.data, lens.ctypes.data, n, out.ctypes.data,
                                               ctypes.byref(st)), "mg_keccak256")
        return [out[32 * i:32 * i + 32].tobytes() for i in range(n)], st.as_dict()


    def valu_peak(self, mul: bool = False) -> Tuple[float, float]:
        ops, ms = ctypes.c_double(0), ctypes.c_double(0)
        _check(self.lib, self.lib.mg_valu_peak(self.handle, 1 if mul else 0, ctypes.byref(ops), ctypes.byref(ms)),
               "mg_valu_peak")
        return ops.value, ms.value


def inflight() -> str:
    """The C-ABI calls in flight on every thread, with the step each is in
    (mg_debug_inflight; for watchdogs: it never blocks), or "" if the
    library is not loaded."""
    if _lib is None:
        return ""
    buf = ctypes.create_string_buffer(8192)
    _lib.mg_debug_inflight(buf, len(buf))
    return buf.value.decode(errors="replace")


def step_times() -> dict:
    """{"call/step": (ms, count)} since the last read (MYTHRIL_AMD_STEP_TIMES=1), then cleared."""
    if _lib is None:
        return {}
    buf = ctypes.create_string_buffer(1 << 16)
    _lib.mg_debug_step_times(buf, len(buf))
    out = {}
    for ln in buf.value.decode(errors="replace").splitlines():
        k, ms, n = ln.rsplit(" ", 2)
        out[k] = (float(ms), int(n))
    return out


def validate(p: Program) -> None:
    lib = load_library()
    d, keep = make_desc(p)
    _check(lib, lib.mg_validate_desc(ctypes.byref(d)), "mg_validate_desc")


def pack_inputs(p: Program, assignments: Sequence[dict]) -> np.ndarray:
    """SoA leaf rows for mg_eval from per-candidate {name: int} dicts."""
    n = len(assignments)
    rows = np.zeros((max(p.n_input_rows, 1), n), dtype=np.uint32)
    for li, node in enumerate(p.leaf_nodes):
        r0, nl = p.input_rows_for(li)
        w = p.leaf_specs[li].width
        for j, a in enumerate(assignments):
            v = int(a.get(node.name, 0)) & ((1 << w) - 1)
            for k in range(nl):
                rows[r0 + k, j] = (v >> (32 * k)) & 0xFFFFFFFF
    return rows


def trace_column(trace: np.ndarray, j: int = 0) -> bytes:
    """Candidate j's trace rows as little-endian bytes (one copy; unpack_one
    reads any node's value from it)."""
    return np.ascontiguousarray(trace[:, j], dtype="<u4").tobytes()


def unpack_one(p: Program, col: bytes, node) -> int:
    """node's traced value in a trace_column."""
    row, cls = p.trace_map[node.id]
    return int.from_bytes(col[4 * row:4 * (row + (8 if cls == "W" else 1))], "little")


def unpack_trace(p: Program, trace: np.ndarray, node) -> List[int]:
    """The traced values of node, one per candidate (trace rows are u32 limbs,
    least significant first)."""
    row, cls = p.trace_map[node.id]
    nl = 8 if cls == "W" else 1
    rows = np.ascontiguousarray(trace[row:row + nl].T, dtype="<u4")   # candidate-major
    return [int.from_bytes(rows[j].tobytes(), "little") for j in range(rows.shape[0])]
