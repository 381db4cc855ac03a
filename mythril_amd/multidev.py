"""Several devices behind one Device interface, in ONE process.

Mythril is a single process, so the drop-in ``get_model`` can
only use more than one GPU if one process drives them all.  ``MultiDevice``
wraps one ``runtime.Device`` context per GPU (``mg_init`` each; one HIP stream
each) and gives the engine the same ``load / search / eval_generated /
keccak256`` surface:

* ``search`` splits the candidate range into rounds; in every round each
  device searches its own contiguous sub-slice of all still-open programs at
  the same time (one host thread per device: ctypes releases the GIL for the
  duration of ``mg_search``).  The per-program witness index is the MIN over
  devices, and rounds run in index order, so the first round with a hit holds
  the global lowest witness; with ``STOP_AFTER_HIT`` that program leaves the
  later rounds, and the search ends when every program has one (the
  between-slices global early stop of SURVEY.md §8(e)).  Exhaustive searches
  (no stop flag) are one round, the range split evenly.
* ``eval_generated`` splits the range over the devices and concatenates.
* programs are replicated: ``load`` uploads to every device (kilobytes).

The torchrun path (one process per GPU, RCCL MIN all-reduce:
``mythril_amd/distributed.py``) stays for ``bench.py``'s scaling runs.
"""
from __future__ import annotations

from concurrent.futures import ThreadPoolExecutor
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import isa

DIV_COUNTS = ("lane_div_steps", "lane_div_full", "lane_div_short", "lane_div_general")   # mg_stats


class MultiProgram:
    """A program loaded on every device."""

    def __init__(self, parts: List, prog):
        self.parts = parts
        self.prog = prog
        self.kernel = None

    def free(self):
        for dp in self.parts:
            dp.free()


class MultiDevice:
    def __init__(self, devices: Sequence, round_size: int = 1 << 22):
        if not devices:
            raise ValueError("MultiDevice needs at least one device")
        self.devs = list(devices)
        self.round_size = round_size
        self.pool = ThreadPoolExecutor(len(self.devs))

    @classmethod
    def open(cls, ids: Sequence[int], **kw) -> "MultiDevice":
        from .runtime import Device
        return cls([Device(i) for i in ids], **kw)

    @property
    def n(self) -> int:
        return len(self.devs)

    def close(self):
        for d in self.devs:
            d.close()
        self.pool.shutdown(wait=True)

    def load(self, p) -> MultiProgram:
        parts = []
        try:
            for d in self.devs:
                parts.append(d.load(p))
        except Exception:
            for dp in parts:
                dp.free()
            raise
        return MultiProgram(parts, p)

    def _split(self, begin: int, count: int) -> List[Tuple[int, int]]:
        base, rem = divmod(count, self.n)
        out, b = [], begin
        for k in range(self.n):
            c = base + (1 if k < rem else 0)
            out.append((b, c))
            b += c
        return out

    def search(self, mps: Sequence[MultiProgram], seed: int, begin: int, count: int,
               flags: int = 0) -> Tuple[List[Optional[int]], dict]:
        found: List[Optional[int]] = [None] * len(mps)
        stats = {"evals": 0, "kernel_ms": 0.0, "launches": 0, "rounds": 0}
        stats.update({k: 0 for k in DIV_COUNTS})
        stop = bool(flags & isa.FLAG_STOP_AFTER_HIT)
        step = self.round_size * self.n if stop else count
        pos, end = begin, begin + count
        while pos < end:
            open_ix = [i for i in range(len(mps)) if found[i] is None]
            if not open_ix:
                break
            n = min(step, end - pos)
            slices = self._split(pos, n)

            def run(k):
                b, c = slices[k]
                if c == 0:
                    return [None] * len(open_ix), {"evals": 0, "kernel_ms": 0.0, "launches": 0}
                return self.devs[k].search([mps[i].parts[k] for i in open_ix], seed, b, c, flags)
            results = list(self.pool.map(run, range(self.n)))
            for j, i in enumerate(open_ix):
                hits = [r[0][j] for r in results if r[0][j] is not None]
                if hits:
                    found[i] = min(hits)
            stats["evals"] += sum(r[1].get("evals", 0) for r in results)
            stats["kernel_ms"] = max(stats["kernel_ms"], 0.0) + max(r[1].get("kernel_ms", 0.0) for r in results)
            stats["launches"] += sum(r[1].get("launches", 0) for r in results)
            for k in DIV_COUNTS:
                stats[k] += sum(r[1].get(k, 0) for r in results)
            stats["rounds"] += 1
            pos += n
            if not stop:
                break
        return found, stats

    def eval_generated(self, mp: MultiProgram, seed: int, begin: int, count: int, trace: bool = True):
        if trace or count < self.n * 256:
            return self.devs[0].eval_generated(mp.parts[0], seed, begin, count, trace)
        slices = self._split(begin, count)
        res = list(self.pool.map(lambda k: self.devs[k].eval_generated(mp.parts[k], seed, *slices[k], trace=False),
                                 range(self.n)))
        return np.concatenate([v for v, _ in res]), None

    def keccak256(self, msgs):
        return self.devs[0].keccak256(msgs)

    def attach_kernel(self, mp: MultiProgram, image: bytes, name: str) -> None:
        for d, dp in zip(self.devs, mp.parts):
            d.attach_kernel(dp, image, name)
        mp.kernel = name
