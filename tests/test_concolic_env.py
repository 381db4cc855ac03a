"""The environment leaves no reference fixture reaches (test_laser_corpus.py
test_leaf_families_covered): TIMESTAMP, GASPRICE, COINBASE, DIFFICULTY in
branch conditions.  SYNTHETIC: a hand-assembled contract (the shape of
tests/testdata/input_contracts/weak_random.sol's block-variable checks, which
has no bytecode in the reference), not reference-derived.  It pins the leaf
names LASER gives these symbols (global_state.py:126-136 new_bitvec:
'{tx}_timestamp', '{tx}_coinbase', '{tx}_block_difficulty'; the transaction's
'gas_price{tx}', transaction/symbolic.py:118-136; environment.block_number,
environment.py:47) and that the engine witnesses every followed successor."""
from mythril_amd.engine import WitnessEngine, prepare
from mythril_amd.ir import Ctx
from tests.fakedev import FakeDevice
from tests.laser_concolic import ACTORS, TxInput, asm as _asm, check_model, run_sequence
from tests.test_engine_cpu import holds


TIMESTAMP, GASPRICE, COINBASE, DIFFICULTY, NUMBER = 0x42, 0x3A, 0x41, 0x44, 0x43
GT, LT, EQ, JUMPI, STOP = 0x11, 0x10, 0x14, 0x57, 0x00

CODE = _asm([
    ("push", 4, 0x60000000), TIMESTAMP, GT, ("ref", "a"), JUMPI, STOP,      # block.timestamp > K
    ("label", "a"), ("push", 1, 0x10), GASPRICE, LT, ("ref", "b"), JUMPI, STOP,   # tx.gasprice < 16
    ("label", "b"), ("push", 20, ACTORS["ATTACKER"]), COINBASE, EQ, ("ref", "c"), JUMPI, STOP,
    ("label", "c"), ("push", 2, 1000), DIFFICULTY, GT, ("ref", "d"), JUMPI, STOP,
    ("label", "d"), ("push", 1, 7), NUMBER, GT, ("ref", "e"), JUMPI, STOP,
    ("label", "e"), STOP,
])


def _run():
    tx = TxInput(b"", sender=ACTORS["ATTACKER"], gas_price=3,
                 env={"timestamp": 0x60000001, "coinbase": ACTORS["ATTACKER"], "block_difficulty": 5000,
                      "block_number": 9})
    return run_sequence(CODE, [tx], balances={x: 10 ** 18 for x in ACTORS.values()})


def test_environment_leaf_names_follow_laser():
    m, run = _run()
    assert run.halts == ["STOP"]
    names = set()
    for q in run.queries:
        for n in q.constraints:
            from mythril_amd.ir import topo
            names |= {x.name for x in topo([n]) if x.op == "var"}
    assert {"1_timestamp", "gas_price1", "1_coinbase", "1_block_difficulty", "block_number"} <= names
    assert sum(q.sat is True for q in run.queries if q.kind == "jumpi") == 5
    # PredictableVars' JUMPI pre hook (dependence_on_predictable_vars.py:68-82) on the
    # TIMESTAMP, COINBASE and NUMBER branches (GASPRICE and DIFFICULTY are not predictable_ops)
    assert sum(q.kind == "PredictableVars/jumpi" for q in run.queries) == 3


def test_environment_queries_witnessed():
    m, run = _run()
    eng = WitnessEngine(dev=FakeDevice(chunk=4096), budget=1 << 14)
    for q in run.queries:
        if not q.sat:
            continue
        assert check_model(q.constraints, run.model)
        (w,) = eng.search([prepare(q.constraints, m.c)])
        assert w is not None and holds(q.constraints, w)
