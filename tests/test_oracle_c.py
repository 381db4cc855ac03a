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
