"""Query.long_program against the oracle.

A long search runs the constraints compiled again into the asm interpreter's
quarter (4 W / 16 N slots, four waves per SIMD) or narrow (24 N slots, three
waves) register layout (engine._quarter_program / _narrow_program): C3's
2.55 G evals/s headline is that program.  Here every such program of the
corpora - C3 and each of the LASER corpus's recompiled queries - gives on
the device, on the kernel of the layout it was compiled for, exactly
oracle/c's verdicts on 2^16 pooled candidates (the same leaf table and pools
as the search program, so the oracle evaluates the same candidates).  The
corpus sweep with the smaller layouts switched off is checked against the
oracle too, not only against the compiled interpreter."""
import json
import os

import numpy as np
import pytest

from mythril_amd import engine
from mythril_amd.engine import DEFAULT_SEED, prepare
from mythril_amd.smt2 import parse_file
from oracle import cdag
from tests.test_gpu_asm import layout_env

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(__file__)
LASER = os.path.join(HERE, "golden", "laser")
SOLVER_LOG = os.path.join(HERE, "golden", "solver_log")
SWEEP = 1 << 16


@pytest.fixture(scope="module")
def dev():
    from mythril_amd.runtime import Device
    d = Device(0)
    yield d
    d.close()


def _queries():
    out = []
    for f in sorted(os.listdir(SOLVER_LOG)):
        s = parse_file(os.path.join(SOLVER_LOG, f))
        out.append((f, prepare(s.asserts, s.ctx)))
    for m in json.load(open(os.path.join(LASER, "manifest.json"))):
        s = parse_file(os.path.join(LASER, m["file"]))
        out.append((m["file"], prepare(s.asserts, s.ctx)))
    return out


@pytest.fixture(scope="module")
def queries():
    return _queries()


def _layout(p):
    w, n = engine._slots_used(p)
    return "quarter" if w <= engine.QUARTER_SLOTS[0] and n <= engine.QUARTER_SLOTS[1] else "narrow"


def test_long_programs_match_the_oracle(dev, queries):
    seen = {"quarter": 0, "narrow": 0}
    c3 = False
    for name, q in queries:
        lp = q.long_program
        if lp is q.program:
            continue
        seen[_layout(lp)] += 1
        c3 = c3 or name.startswith("c3")
        _, _, vo = cdag.evaluate(q.lowered.conjuncts, DEFAULT_SEED, 0, SWEEP, want_verdict=True,
                                 specs=cdag.program_specs(lp))
        dl = dev.load(lp)
        try:
            assert dev.engine_of(dl) == "asm", name
            vl, _ = dev.eval_generated(dl, DEFAULT_SEED, 0, SWEEP, trace=False)
        finally:
            dl.free()
        assert np.array_equal(vl.astype(np.uint8), vo), (name, _layout(lp), int(np.count_nonzero(vl != vo)))
    print(f"long programs checked against oracle/c: {seen}")
    assert c3, "C3's long program (the narrow layout) is covered"
    assert seen["quarter"] >= 50 and seen["narrow"] >= 5, seen


@pytest.mark.parametrize("env", [{"MYTHRIL_AMD_ASM_QUARTER": "0"}, {"MYTHRIL_AMD_ASM_NARROW": "0"}])
def test_wider_layouts_match_the_oracle(dev, queries, env):
    """The programs a smaller layout would take, on the wider kernels: oracle/c's verdicts."""
    n = 1 << 14
    for name, q in queries[::5]:
        _, _, vo = cdag.evaluate(q.lowered.conjuncts, DEFAULT_SEED, 0, n, want_verdict=True,
                                 specs=cdag.program_specs(q.program))
        with layout_env(**env):
            dp = dev.load(q.program)
        try:
            v, _ = dev.eval_generated(dp, DEFAULT_SEED, 0, n, trace=False)
        finally:
            dp.free()
        assert np.array_equal(v.astype(np.uint8), vo), (name, env)
