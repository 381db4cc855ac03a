"""The LASER-shaped corpus over the reference's bytecode (tests/golden/laser)
on gfx950:

* verdict sweep: 2^16 pooled candidates of every query on the device
  interpreter equal the C oracle's (oracle/c) on the same indices;
* search at config C2's count (2^24 candidates per query, early exit +
  stop-after-hit, 64 programs per launch): every witness satisfies the
  ORIGINAL formula under the oracle (arrays and UFs included), and every SAT
  query (satisfied by the concolic model) is witnessed."""
import json
import os

import numpy as np
import pytest

from mythril_amd.engine import DEFAULT_SEED, WitnessEngine, prepare
from mythril_amd.smt2 import parse_file
from oracle import cdag
from tests.test_engine_cpu import holds

pytestmark = pytest.mark.gpu

CORPUS = os.path.join(os.path.dirname(__file__), "golden", "laser")
MANIFEST = json.load(open(os.path.join(CORPUS, "manifest.json")))


@pytest.fixture(scope="module")
def queries():
    out = []
    for m in MANIFEST:
        s = parse_file(os.path.join(CORPUS, m["file"]))
        out.append((m, s, prepare(s.asserts, s.ctx)))
    return out


@pytest.fixture(scope="module")
def eng():
    e = WitnessEngine(device=0, budget=1 << 24, op_budget=None)
    yield e
    e.close()


def test_verdict_sweep_matches_oracle(queries, eng):
    n = 1 << 16
    for m, s, q in queries:
        _, _, vo = cdag.evaluate(q.lowered.conjuncts, DEFAULT_SEED, 0, n, want_verdict=True,
                                 specs=cdag.program_specs(q.program))
        dp = eng.dev.load(q.program)
        vi, _ = eng.dev.eval_generated(dp, DEFAULT_SEED, 0, n, trace=False)
        dp.free()
        assert np.array_equal(vi.astype(np.uint8), vo), m["file"]


def test_search_at_c2_count(queries, eng):
    found = {"sat": 0, "unknown": 0}
    total = {"sat": 0, "unknown": 0}
    missed = []
    for i in range(0, len(queries), 64):
        chunk = queries[i:i + 64]
        ws = eng.search([q for _, _, q in chunk], count=1 << 24)
        for (m, s, q), w in zip(chunk, ws):
            total[m["status"]] += 1
            if w is not None:
                assert holds(s.asserts, w), m["file"]
                found[m["status"]] += 1
            elif m["status"] == "sat":
                missed.append(m["file"])
    print(f"LASER corpus at 2^24: witnessed {found} of {total}; SAT missed: {missed}")
    # every query the concolic run satisfied is witnessed (VERDICT r2 item 5:
    # the calldatasize pools now lead with the highest guard of a calldata read)
    assert found["sat"] == total["sat"], (found, total, missed)
