"""The C restatement (oracle/c, used for the CPU baseline and large sweeps)
agrees with the Python oracle on random DAGs and on the VMTests DAGs."""
import json
import os

import pytest

from mythril_amd.compiler import compile_program
from oracle import cdag
from oracle.dag_eval import eval_nodes
from oracle.vmtest_runner import run_case
from tests.helpers import RandDag, oracle_models


@pytest.fixture(scope="module", autouse=True)
def built():
    cdag.subprocess_build()


@pytest.mark.parametrize("seed", range(25))
def test_c_oracle_matches_python_oracle(seed):
    dag = RandDag(500 + seed)
    conj = [dag.boolean(4) for _ in range(3)]
    p = compile_program(conj)
    _, _, v = cdag.evaluate(conj, 99, 1 << 33, 48, want_verdict=True)
    for j, m in enumerate(oracle_models(p, 99, 1 << 33, 48)):
        vals = eval_nodes(conj, m)
        assert v[j] == int(all(vals[c.id] for c in conj))


def test_c_oracle_first_witness_matches_scan():
    dag = RandDag(4, widths=[8])
    x = dag.ctx.var("x", 8)
    conj = [dag.ctx.app("=", x, dag.ctx.const(0x5A, 8))]
    tot, first, v = cdag.evaluate(conj, 5, 0, 5000, want_verdict=True)
    assert tot == int(v.sum()) and tot > 0
    assert first == int(next(i for i in range(5000) if v[i]))


def _pooled_query(name):
    from mythril_amd.engine import prepare
    from mythril_amd.smt2 import parse_file
    s = parse_file(os.path.join(os.path.dirname(__file__), "golden", "solver_log", name))
    return prepare(s.asserts, s.ctx)


@pytest.mark.parametrize("name", ["c2_token_transfer_ok.smt2", "c4_wallet_onlyowner.smt2"])
def test_c_oracle_pool_leaves_match_python_oracle(name):
    """Pool-driven candidates (interleaved / hashed digits, RANDOM entries) in the
    C oracle agree with oracle/philox.py leaf_value + the Python evaluator."""
    q = _pooled_query(name)
    p = q.program
    conj = q.lowered.conjuncts
    specs = cdag.program_specs(p)
    assert any(sp["pool"] for sp in specs.values())
    tot, first, v = cdag.evaluate(conj, 0x5EED0001, 0, 256, want_verdict=True, specs=specs)
    models = oracle_models(p, 0x5EED0001, 0, 256)
    want = [int(all(eval_nodes(conj, m)[c.id] for c in conj)) for m in models]
    assert list(map(int, v)) == want
    assert tot == sum(want) and tot > 0


def test_c_oracle_pool_leaves_match_host_emulator():
    """C3 (BECToken overflow; 2 185 conjuncts, pooled calldata words): the C
    oracle's verdicts equal the interpreter's host build on 4 096 candidates."""
    from tests.helpers import emu_eval
    q = _pooled_query("c3_bec_batchtransfer_overflow.smt2")
    n = 4096
    _, _, v = cdag.evaluate(q.lowered.conjuncts, 0x5EED0001, 0, n, want_verdict=True,
                            specs=cdag.program_specs(q.program))
    e, _ = emu_eval(q.program, None, n, seed=0x5EED0001, begin=0)
    assert (v.astype(int) == e.astype(int)).all()
    assert 0 < int(v.sum()) < n
