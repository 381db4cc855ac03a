"""Test-only device double: the engine's Device interface on the host emulator
(the same interpreter source as the gfx950 kernels), so engine/drop-in logic is
exercised on CPU.  Never used by the product."""
import numpy as np

from tests.helpers import emu_eval


class _DP:
    def __init__(self, p):
        self.prog = p
        self.handle = 1

    def free(self):
        pass


class FakeDevice:
    def __init__(self, chunk=1 << 12):
        self.chunk = chunk

    def load(self, p):
        return _DP(p)

    def search(self, dps, seed, begin, count, flags=0):
        out = []
        evals = 0
        for dp in dps:
            found = None
            pos = begin
            while pos < begin + count:
                n = min(self.chunk, begin + count - pos)
                v, _ = emu_eval(dp.prog, None, n, seed=seed, begin=pos)
                evals += n
                nz = np.nonzero(v)[0]
                if nz.size:
                    found = pos + int(nz[0])
                    break
                pos += n
            out.append(found)
        return out, {"evals": evals, "kernel_ms": 0.0}

    def search_begin(self, dps, seed, begin, count, flags=0):
        """Device.search_begin on the host build: the search runs at the end."""
        assert getattr(self, "_begun", None) is None, "a search is pending"
        self._begun = (list(dps), seed, begin, count, flags)
        self.begin_calls = getattr(self, "begin_calls", 0) + 1

    def search_end(self, witness=None):
        """Device.search_end: the search, then each witness program evaluated
        at its program's index (the trace column), as mg_search_end does."""
        dps, seed, begin, count, flags = self._begun
        self._begun = None
        found, st = self.search(dps, seed, begin, count, flags)
        traces = [None] * len(dps)
        if witness is not None:
            for i, (p, f) in enumerate(zip(witness, found)):
                if p is not None and f is not None and p.n_trace_rows:
                    _, tr = emu_eval(p, None, 1, seed=seed, begin=f)
                    traces[i] = tr
        return found, st, traces

    def eval_generated(self, dp, seed, begin, count, trace=True):
        return emu_eval(dp.prog, None, count, seed=seed, begin=begin)

    def witness_leaves(self, dp, seed, index):
        """Device.witness_leaves (mg_witness_leaves) on the host build of the
        same leaf generator (mw_leaf.h, mwh_leaf_values)."""
        import ctypes

        from mythril_amd.runtime import make_desc
        from tests.helpers import host_emu
        p = dp.prog
        d, keep = make_desc(p)
        out = np.zeros(max(1, len(p.leaf_nodes)) * 8, dtype=np.uint32)
        f = host_emu().mwh_leaf_values
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p]
        rc = f(ctypes.byref(d), seed & ((1 << 64) - 1), index, out.ctypes.data)
        assert rc == 0
        self.witness_leaf_calls = getattr(self, "witness_leaf_calls", 0) + 1
        vals = []
        for i, node in enumerate(p.leaf_nodes):
            v = sum(int(out[8 * i + k]) << (32 * k) for k in range(8))
            vals.append(v & ((1 << (1 if node.width == 0 else node.width)) - 1))
        return vals

    def keccak256(self, msgs):
        """Device.keccak256 on the host build of the same Keccak source."""
        from tests.helpers import host_emu
        self.keccak_launches = getattr(self, "keccak_launches", 0) + 1
        data = b"".join(msgs) or b"\0"
        off = np.zeros(len(msgs), dtype=np.uint64)
        if len(msgs) > 1:
            off[1:] = np.cumsum([len(m) for m in msgs[:-1]])
        ln = np.array([len(m) for m in msgs], dtype=np.uint32)
        out = np.zeros(32 * len(msgs), dtype=np.uint8)
        host_emu().mwh_keccak256(data, off.ctypes.data, ln.ctypes.data, len(msgs), out.ctypes.data)
        return [out[32 * i:32 * i + 32].tobytes() for i in range(len(msgs))], {}

    def close(self):
        pass
