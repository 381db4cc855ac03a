"""The --solver-log corpus (C2-C4 shapes, tests/golden/solver_log) replayed on
the MI355X through the C-ABI: the same expectations as tests/test_replay.py
(witness for every SAT query, valid on the original formula under the oracle;
never one for an UNSAT query), all queries in one launch."""
import pytest

from mythril_amd.engine import WitnessEngine
from mythril_amd.replay import replay
from tests.test_replay import CORPUS, check

pytestmark = pytest.mark.gpu


def test_replay_corpus_on_device():
    eng = WitnessEngine(device=0, seed=0x5EED0002, budget=1 << 20)
    try:
        res = replay(CORPUS, eng)
        check(res, "device, 2^20 candidates")
        assert eng.stats["searches"] == 1
    finally:
        eng.close()
