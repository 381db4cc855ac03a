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

    def eval_generated(self, dp, seed, begin, count, trace=True):
        return emu_eval(dp.prog, None, count, seed=seed, begin=begin)

    def close(self):
        pass
