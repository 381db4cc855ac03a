"""Replay of the --solver-log corpus (tests/golden/solver_log, C2-C4 shapes):
sat queries yield witnesses that satisfy the ORIGINAL formula (oracle), unsat
ones never do, objective queries stay with z3.  CPU: host emulator behind a
fake device; tests/test_gpu_replay.py runs the same on the MI355X."""
import glob
import os

import pytest

from mythril_amd.replay import replay
from mythril_amd.smt2 import parse_file, to_smt2
from oracle.dag_eval import ArrayVal, eval_nodes

CORPUS = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "solver_log", "*.smt2")))


def expectation(path):
    return open(path).readline().split(":")[1].strip()


def check(results, budget_note=""):
    assert len(results) == len(CORPUS)
    for r in results:
        exp = expectation(r.path)
        if exp == "unsat":
            assert r.status == "miss", (r.path, r.status)
        else:
            assert r.status == "witness", (r.path, r.status, budget_note)
            # the witness extends to a model of the ORIGINAL (un-lowered) formula
            s = parse_file(r.path)
            model = dict(r.values)
            for name, cells in r.arrays.items():
                model[name] = ArrayVal(cells)
            for name, points in r.functions.items():
                model[name] = (points, 0)
            vals = eval_nodes(s.asserts, model)
            assert all(vals[a.id] for a in s.asserts), r.path


def engine(dev=None, budget=1 << 16):
    from mythril_amd.engine import WitnessEngine
    if dev is None:
        from tests.fakedev import FakeDevice
        dev = FakeDevice(chunk=4096)
    return WitnessEngine(dev=dev, seed=0x5EED0002, budget=budget)


def test_corpus_is_present_and_parses():
    assert len(CORPUS) >= 7
    for p in CORPUS:
        s = parse_file(p)
        assert s.asserts and not s.minimize


def test_replay_corpus_on_host_emulator():
    """Every SAT query of the corpus (C2 token transfer, C3 BECToken
    batchTransfer overflow, C4 wallet onlyowner) is witnessed within 2^16
    candidates; the UNSAT ones never are (pools.py domain restriction and
    word-tied calldata bytes)."""
    check(replay(CORPUS, engine()))


def test_objective_queries_stay_with_z3(tmp_path):
    s = parse_file(CORPUS[0])
    f = tmp_path / "opt.smt2"
    f.write_text(to_smt2(s.asserts, minimize=[s.ctx.var("1_calldatasize", 256)]))
    (r,) = replay([str(f)], engine())
    assert r.status == "z3"


def test_unsupported_formula_falls_back(tmp_path):
    f = tmp_path / "bad.smt2"
    f.write_text("(declare-fun x () Int)\n(assert (> x 1))\n")
    (r,) = replay([str(f)], engine())
    assert r.status == "unsupported"
