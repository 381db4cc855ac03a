"""mg_eval_program (round 6): one library call uploads,
evaluates and releases a program that is not kept - the witness program a
hit reads once - with exactly the verdicts and trace rows of mg_prog_load +
mg_eval_generated + mg_prog_free, on the asm interpreter (witness programs)
and on the compiled interpreter (a program with more wide divisions than the
asm engines take)."""
import json
import os

import numpy as np
import pytest

from mythril_amd.compiler import compile_program
from mythril_amd.engine import DEFAULT_SEED, prepare
from mythril_amd.smt2 import parse_file

pytestmark = pytest.mark.gpu

CORPUS = os.path.join(os.path.dirname(__file__), "golden", "laser")


@pytest.fixture(scope="module")
def dev():
    from mythril_amd.runtime import Device
    d = Device(0)
    yield d
    d.close()


def _both(dev, p, begin, n):
    v1, t1 = dev.eval_program(p, DEFAULT_SEED, begin, n)
    dp = dev.load(p)
    try:
        v2, t2 = dev.eval_generated(dp, DEFAULT_SEED, begin, n)
        engine = dev.engine_of(dp)
    finally:
        dp.free()
    return v1, t1, v2, t2, engine


def test_witness_programs_one_shot(dev):
    man = json.load(open(os.path.join(CORPUS, "manifest.json")))
    engines = set()
    for m in man[::17]:
        s = parse_file(os.path.join(CORPUS, m["file"]))
        q = prepare(s.asserts, s.ctx)
        p = q.trace_program
        for begin, n in ((0, 1), (12345, 1), (0, 300)):
            v1, t1, v2, t2, engine = _both(dev, p, begin, n)
            engines.add(engine)
            assert np.array_equal(v1, v2), m["file"]
            assert (t1 is None and t2 is None) or np.array_equal(t1, t2), (m["file"], begin, n)
    assert "asm" in engines


def test_compiled_interpreter_one_shot(dev):
    from tests.test_divcount import _division_dag
    p = compile_program(_division_dag(), trace=[])
    v1, _, v2, _, engine = _both(dev, p, 7, 4096)
    assert engine == "interp" and np.array_equal(v1, v2)


def test_many_one_shots_reuse_the_pool(dev):
    """Each call's buffer goes back to the context's pool: 2 000 calls run in
    the memory of one."""
    s = parse_file(os.path.join(CORPUS, json.load(open(os.path.join(CORPUS, "manifest.json")))[0]["file"]))
    p = prepare(s.asserts, s.ctx).trace_program
    first = dev.eval_program(p, DEFAULT_SEED, 99, 1)
    for _ in range(2000):
        v, t = dev.eval_program(p, DEFAULT_SEED, 99, 1)
    assert np.array_equal(v, first[0]) and (t is None or np.array_equal(t, first[1]))
