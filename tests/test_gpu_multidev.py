"""Single-process multi-device search on the GPU (mythril_amd/multidev.py): two
contexts on the box's device behave as two GPUs (own streams, concurrent
launches from two host threads) and must give exactly one context's witness
indices and verdicts."""
import os

import numpy as np
import pytest

from mythril_amd import isa
from mythril_amd.engine import DEFAULT_SEED, prepare
from mythril_amd.smt2 import parse_file

pytestmark = pytest.mark.gpu

LOG = os.path.join(os.path.dirname(__file__), "golden", "solver_log")


def test_two_contexts_match_one():
    from mythril_amd.multidev import MultiDevice
    from mythril_amd.runtime import Device
    qs = []
    for f in sorted(os.listdir(LOG)):
        s = parse_file(os.path.join(LOG, f))
        qs.append(prepare(s.asserts, s.ctx))
    one = Device(0)
    md = MultiDevice([Device(0), Device(0)], round_size=1 << 16)
    try:
        flags = isa.FLAG_EARLY_EXIT | isa.FLAG_STOP_AFTER_HIT
        ones = [one.load(q.program) for q in qs]
        want, _ = one.search(ones, DEFAULT_SEED, 0, 1 << 20, flags)
        mps = [md.load(q.program) for q in qs]
        got, st = md.search(mps, DEFAULT_SEED, 0, 1 << 20, flags)
        assert got == want and any(w is not None for w in want) and any(w is None for w in want)
        ex_want, _ = one.search(ones, DEFAULT_SEED, 0, 1 << 18, 0)
        ex_got, st = md.search(mps, DEFAULT_SEED, 0, 1 << 18, 0)
        assert ex_got == ex_want and st["evals"] == len(qs) * (1 << 18)
        v1, _ = one.eval_generated(ones[0], DEFAULT_SEED, 0, 1 << 14, trace=False)
        v2, _ = md.eval_generated(mps[0], DEFAULT_SEED, 0, 1 << 14, trace=False)
        assert np.array_equal(v1, v2)
        for mp in mps:
            mp.free()
    finally:
        md.close()   # frees any program still loaded before the context
        one.close()
