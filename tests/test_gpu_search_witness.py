"""mg_search_begin / mg_search_end (round 6): the witness
read in the search's own synchronisation.

* begin + end give the same lowest indices and statistics as mg_search, and
  each witness trace equals mg_eval_program's of the same witness program at
  the found index (LASER corpus, 64 programs per launch);
* the engine's answers (indices and witness values) are the same with the
  witness in the launch and without (MYTHRIL_AMD_WITNESS_IN_LAUNCH=0);
* while a search is pending, calls that launch work on the context are
  refused, uploads are allowed, and freeing one of its programs waits for it."""
import json
import os

import numpy as np
import pytest

from mythril_amd import engine, isa
from mythril_amd.engine import DEFAULT_SEED, WitnessEngine, prepare
from mythril_amd.runtime import EngineError
from mythril_amd.smt2 import parse_file

pytestmark = pytest.mark.gpu

CORPUS = os.path.join(os.path.dirname(__file__), "golden", "laser")
FLAGS = isa.FLAG_EARLY_EXIT | isa.FLAG_STOP_AFTER_HIT


@pytest.fixture(scope="module")
def eng():
    e = WitnessEngine(device=0)
    yield e
    e.close()


@pytest.fixture(scope="module")
def queries():
    out = []
    for m in json.load(open(os.path.join(CORPUS, "manifest.json")))[::6]:
        s = parse_file(os.path.join(CORPUS, m["file"]))
        out.append((m["file"], s, prepare(s.asserts, s.ctx)))
    return out


def test_begin_end_equals_search_and_eval(eng, queries):
    dev = eng.dev
    qs = [q for _, _, q in queries][:64]
    dps = [dev.load(q.program) for q in qs]
    try:
        (ref, st_ref) = dev.search(dps, DEFAULT_SEED, 0, 1 << 16, FLAGS)
        dev.search_begin(dps, DEFAULT_SEED, 0, 1 << 16, FLAGS)
        wps = [q.trace_program for q in qs]
        found, st, traces = dev.search_end(wps)
        assert found == ref
        assert st["evals"] > 0
        hits = 0
        for q, p, f, tr in zip(qs, wps, found, traces):
            if f is None:
                assert tr is None
                continue
            assert tr is not None
            _, want = dev.eval_program(p, DEFAULT_SEED, f, 1)
            assert np.array_equal(tr[:, 0], want[:, 0])
            hits += 1
        assert hits >= 10
        # without witness programs: only the search
        dev.search_begin(dps, DEFAULT_SEED, 0, 1 << 16, FLAGS)
        f2, _, t2 = dev.search_end(None)
        assert f2 == ref and all(t is None for t in t2)
    finally:
        for dp in dps:
            dp.free()


def test_engine_same_witnesses_either_way(eng, queries, monkeypatch):
    qs = [q for _, _, q in queries]
    a = eng.search(qs)
    monkeypatch.setattr(engine, "WITNESS_IN_LAUNCH", False)
    b = eng.search(qs)
    assert [w and w.index for w in a] == [w and w.index for w in b]
    for wa, wb in zip(a, b):
        if wa is not None:
            assert wa.values == wb.values and wa.arrays == wb.arrays and wa.functions == wb.functions


def test_pending_search_guards(eng, queries):
    dev = eng.dev
    q = queries[0][2]
    dp, dp2 = dev.load(q.program), dev.load(q.program)
    try:
        dev.search_begin([dp, dp2], DEFAULT_SEED, 0, 1 << 20, 0)
        for call in (lambda: dev.search([dp], DEFAULT_SEED, 0, 256, 0),
                     lambda: dev.eval_generated(dp, DEFAULT_SEED, 0, 4),
                     lambda: dev.eval_program(q.program, DEFAULT_SEED, 0, 1),
                     lambda: dev.search_begin([dp], DEFAULT_SEED, 0, 256, 0)):
            with pytest.raises(EngineError):
                call()
        extra = dev.load(q.program)       # uploads are allowed meanwhile
        dp2.free()                         # waits for the pending search
        found, st, _ = dev.search_end(None)
        assert st["evals"] == 2 * (1 << 20)
        (ref,), _ = dev.search([dp], DEFAULT_SEED, 0, 1 << 20, 0)
        assert found[0] == ref == found[1]
        extra.free()
        with pytest.raises(EngineError):   # nothing pending any more
            dev.search_end(None)
    finally:
        dp.free()
