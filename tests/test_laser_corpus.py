"""The LASER-shaped corpus derived from the reference's bytecode fixtures
(tests/golden/laser, made by tools/make_laser_corpus.py over
tests/laser_concolic.py).

CPU checks: the committed files are exactly what the generator produces
(deterministic; one scenario re-run here), every query lowers to the engine's
vocabulary, and every witness the engine finds on the host build of the
interpreter satisfies the ORIGINAL formula under the oracle.
tests/test_gpu_laser.py runs the same corpus on the device at C2's 2^24."""
import gzip
import json
import os
import sys

import pytest

from mythril_amd.compiler import Unsupported
from mythril_amd.engine import WitnessEngine, prepare
from mythril_amd.smt2 import parse_file
from tests.fakedev import FakeDevice
from tests.test_engine_cpu import holds

HERE = os.path.dirname(os.path.abspath(__file__))
CORPUS = os.path.join(HERE, "golden", "laser")
MANIFEST = json.load(open(os.path.join(CORPUS, "manifest.json")))


def test_manifest_matches_files():
    files = {f for f in os.listdir(CORPUS) if f.endswith(".smt2.gz")}
    assert files == {m["file"] for m in MANIFEST}
    assert len(MANIFEST) >= 100
    contracts = {m["contract"] for m in MANIFEST}
    # all 17 reference .sol.o fixtures (tests/testdata/inputs), two VMTests, one synthetic
    assert contracts == {"underflow", "overflow", "metacoin", "suicide", "flag_array", "origin", "calls",
                         "kinds_of_calls", "returnvalue", "ether_send", "exceptions_0.8.0", "environments",
                         "exceptions", "multi_contracts", "nonascii", "safe_funcs", "symbolic_exec_bytecode",
                         "vm:vmIOandFlowOperations/DynamicJumpJD_DependsOnJumps0",
                         "vm:vmIOandFlowOperations/DynamicJumpJD_DependsOnJumps1", "synthetic:predictable"}
    assert sum(m["status"] == "sat" for m in MANIFEST) >= 390
    kinds = {m["kind"] for m in MANIFEST}
    # every feasibility caller of SURVEY §8a A10 and the modules whose
    # get_transaction_sequence sets the reference's issue tests pin
    assert {"jumpi", "EtherThief", "StateChangeAfterCall/external_call", "StateChangeAfterCall/attacker_callee",
            "StateChangeAfterCall/balance_change", "IntegerArithmetics/addition",
            "IntegerArithmetics/subtraction", "IntegerArithmetics/multiplication",
            "MutationPruner", "DependencyPruner", "ExternalCalls/precompile", "ExternalCalls/user_supplied",
            "PredictableVars/blockhash", "PredictableVars/jumpi", "Exceptions",
            "AccidentallyKillable/attacker_beneficiary", "AccidentallyKillable/any_sender"} <= kinds
    # DependencyPruner's queries are tuples: no keccak conditions (model.py:35-36)
    for m in MANIFEST:
        assert m["tuple"] == (m["kind"] == "DependencyPruner"), m["file"]
        if m["tuple"]:
            assert "keccak256_512-1" not in gzip.open(os.path.join(CORPUS, m["file"]), "rt").read()
    # multi-transaction sets carry one sender-among-actors constraint per transaction
    last = max(MANIFEST, key=lambda m: (m["tx"], m["conjuncts"]))
    text = gzip.open(os.path.join(CORPUS, last["file"]), "rt").read()
    for t in range(1, last["tx"] + 1):
        assert f"(= |sender_{t}| #x000000000000000000000000deadbeef" in text


def test_generator_is_deterministic(tmp_path):
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))
    from make_laser_corpus import write
    made = write(str(tmp_path), only="suicide/t2_kill")
    assert made
    for m in made:
        a = open(os.path.join(tmp_path, m["file"]), "rb").read()
        b = open(os.path.join(CORPUS, m["file"]), "rb").read()
        assert a == b, m["file"]


def test_every_query_lowers():
    for m in MANIFEST:
        s = parse_file(os.path.join(CORPUS, m["file"]))
        try:
            prepare(s.asserts, s.ctx)
        except Unsupported as e:   # pragma: no cover - a regression
            pytest.fail(f"{m['file']}: {e}")


def test_host_witnesses_are_sound():
    eng = WitnessEngine(dev=FakeDevice(chunk=4096), seed=0x5EED0002, budget=1 << 12)
    found = {"sat": 0, "unknown": 0}
    for m in MANIFEST:
        s = parse_file(os.path.join(CORPUS, m["file"]))
        q = prepare(s.asserts, s.ctx)
        (w,) = eng.search([q])
        if w is not None:
            assert holds(s.asserts, w), m["file"]
            found[m["status"]] += 1
    assert found["sat"] >= 40, found


def _declared(m):
    import re
    return set(re.findall(r"\(declare-fun \|([^|]+)\|", gzip.open(os.path.join(CORPUS, m["file"]), "rt").read()))


def test_leaf_families_covered():
    """The leaf schema as the reference's own bytecode reaches
    it: every family below appears in a committed query.  TIMESTAMP, COINBASE,
    DIFFICULTY and GASPRICE reach no branch in any reference fixture (their
    opcode bytes occur only inside the .sol.o metadata, or in VMTests without
    a JUMPI; weak_random.sol has no bytecode), so those leaves are exercised by
    the synthetic scenario in tests/test_concolic_env.py instead."""
    import re
    fams = set()
    for m in MANIFEST:
        for n in _declared(m):
            n = re.sub(r"^\d+_", "{tx}_", n)
            n = re.sub(r"_\d+$|\d+$", "", n)
            fams.add(re.sub(r"^Storage.*", "Storage", n))
    for fam in ("sender", "call_value", "{tx}_calldatasize", "{tx}_calldata", "balance", "Storage",
                "{tx}_retval", "{tx}_gas", "block_number", "keccak256", "Power"):
        assert fam in fams, (fam, sorted(fams))


def test_ether_thief_query_pinned_by_reference_calldata():
    """tests/integration_tests/analysis_tests.py:9-19: myth analyze of
    flag_array.sol.o -t 1 -m EtherThief reports one issue whose transaction 1
    input is 0xab125858...04d2 (extractMoney(1234)).  The EtherThief get_model
    query of that path (ether_thief.py:60-76: the attacker's balance above its
    starting balance, sender == ATTACKER, caller == origin) is satisfied by the
    model whose calldata is exactly that input, and the search finds a witness
    that satisfies it under the oracle."""
    from tests.laser_concolic import run_sequence, ACTORS
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))
    from make_laser_corpus import SCENARIOS, load_code
    name, txs = SCENARIOS["flag_array"][0][:2]
    assert name == "t2_extract_money"
    expected = "0xab12585800000000000000000000000000000000000000000000000000000000000004d2"
    assert "0x" + txs[1].calldata.hex() == expected
    m, run = run_sequence(load_code("flag_array"), txs, balances={x: 10 ** 18 for x in ACTORS.values()})
    thief = [q for q in run.queries if q.kind == "EtherThief"]
    assert len(thief) == 1 and thief[0].sat
    calldata = run.model["2_calldata"]
    assert bytes(calldata.get(i) for i in range(len(txs[1].calldata))) == bytes.fromhex(expected[2:])
    mf = [x for x in MANIFEST if x["contract"] == "flag_array" and x["kind"] == "EtherThief"]
    assert len(mf) == 1 and mf[0]["status"] == "sat"
    s = parse_file(os.path.join(CORPUS, mf[0]["file"]))
    q = prepare(s.asserts, s.ctx)
    eng = WitnessEngine(dev=FakeDevice(chunk=4096), budget=1 << 16)
    (w,) = eng.search([q])
    assert w is not None and holds(s.asserts, w)
    idx = sum(w.arrays["2_calldata"].get(i, 0) << (8 * (35 - i)) for i in range(4, 36))
    assert idx == 1234           # the only flagged index: the witness's calldata is the reference's


def _run(contract, scenario):
    from tests.laser_concolic import run_sequence
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))
    from make_laser_corpus import SCENARIOS, load_code, scenario_balances
    for name, txs, *opt in SCENARIOS[contract]:
        if name == scenario:
            opts = opt[0] if opt else {}
            return txs, run_sequence(load_code(contract), txs, storage=opts.get("storage"),
                                     balances=scenario_balances(opts))[1]
    raise KeyError(scenario)


def test_exceptions_issues_pinned_by_reference():
    """tests/integration_tests/analysis_tests.py:21-31: myth analyze of
    exceptions_0.8.0.sol.o -t 1 -m Exceptions reports TWO issues.  With one
    message call after the creation, the paths that reach an assertion
    failure (a Panic(0x01) REVERT, exceptions.py:58-84) are assert1() and
    fail() (val is still 0); change_val() reaches none.  The constraint set
    the module hands to get_transaction_sequence at each is satisfied by the
    concrete model (and witnessed on the device, test_gpu_laser.py)."""
    issues = {}
    for scen in ("t2_assert_fails", "t2_fail", "t2_change_val"):
        txs, run = _run("exceptions_0.8.0", scen)
        assert len(txs) == 2 and txs[0].creation        # -t 1: the creation, then one message call
        exc = [q for q in run.queries if q.kind == "Exceptions"]
        issues[scen] = len(exc)
        assert all(q.sat and q.tx == 2 for q in exc), scen
    assert issues == {"t2_assert_fails": 1, "t2_fail": 1, "t2_change_val": 0}
    mf = [m for m in MANIFEST if m["contract"] == "exceptions_0.8.0" and m["kind"] == "Exceptions"
          and m["scenario"] in ("t2_assert_fails", "t2_fail")]
    assert len(mf) == 2 and all(m["status"] == "sat" for m in mf)


def test_accidentally_killable_issue_pinned_by_reference():
    """analysis_tests.py:32-41: myth analyze of symbolic_exec_bytecode.sol.o -t 1
    -m AccidentallyKillable reports ONE issue.  The creation takes a symbolic
    constructor argument (the creation calldata behind CODESIZE / CODECOPY,
    instructions.py:977-993,1065-1130) that becomes an immutable of the
    runtime code; commencekilling() then self-destructs to msg.sender.  The
    module's first constraint set (suicide.py:70-80: world + [to == ATTACKER]
    + the sender conditions) is satisfiable, so the issue is the
    'attacker_beneficiary' one, and it is the only SELFDESTRUCT query."""
    txs, run = _run("symbolic_exec_bytecode", "t2_commence_killing")
    assert len(txs) == 2 and txs[0].creation
    kill = [q for q in run.queries if q.kind.startswith("AccidentallyKillable")]
    assert [(q.kind, q.sat) for q in kill] == [("AccidentallyKillable/attacker_beneficiary", True)]
    mf = [m for m in MANIFEST if m["contract"] == "symbolic_exec_bytecode"
          and m["scenario"] == "t2_commence_killing" and m["kind"].startswith("AccidentallyKillable")]
    assert len(mf) == 1 and mf[0]["status"] == "sat"
    # the immutable is symbolic in the runtime code: getBytes compares against it
    txs, run = _run("symbolic_exec_bytecode", "t2_get_bytes")
    from mythril_amd.ir import topo
    assert any(n.op == "bvshl" for q in run.queries if q.tx == 2 for n in topo(q.constraints))


def test_pruners_follow_the_reference():
    """MutationPruner asks world + [callvalue >u 0] at every message call's end
    (mutation_pruner.py:60-86); DependencyPruner's tuples compare a location
    written in the previous transaction with one read on a path through the
    revisited block (dependency_pruner.py:146-200), and a path whose previous
    transaction wrote nothing is pruned (metacoin's third call)."""
    txs, run = _run("underflow", "t3_send_send_balance")
    assert sum(q.kind == "MutationPruner" for q in run.queries) == 3
    dep = [q for q in run.queries if q.kind == "DependencyPruner"]
    assert dep and all(q.tuple_form and len(q.constraints) == 1 and q.constraints[0].op == "=" for q in dep)
    assert all(q.tx == 3 for q in dep)
    _, run = _run("metacoin", "t3_sendtoken")
    assert run.halts[2] == "PRUNED"


def _ground_truth():
    return json.loads(gzip.open(os.path.join(HERE, "golden", "laser_ground_truth.json.gz"), "rt").read())


def test_ground_truth_witnesses_hold():
    """every "unknown" query the device witnessed (up to
    2^32 candidates, tools/ground_truth.py, profiles/r5a) is SAT: its recorded
    witness satisfies the ORIGINAL formula under the oracle (arrays and UF
    tables included), re-checked here without a GPU."""
    from oracle.dag_eval import ArrayVal, eval_nodes
    gt = _ground_truth()
    unknown = {m["file"] for m in MANIFEST if m["status"] == "unknown"}
    assert set(gt["witnessed"]) | set(gt["no_witness"]) == unknown
    for f, w in gt["witnessed"].items():
        s = parse_file(os.path.join(CORPUS, f))
        model = {k: int(v, 16) for k, v in w["values"].items()}
        for name, cells in w["arrays"].items():
            model[name] = ArrayVal({int(i, 16): int(v, 16) for i, v in cells.items()})
        for name, table in w["functions"].items():
            model[name] = ({tuple(int(a, 16) for a in args): int(v, 16) for args, v in table}, 0)
        vals = eval_nodes(s.asserts, model)
        assert all(vals[x.id] for x in s.asserts), f


def test_unwitnessed_queries_have_reasons():
    """The rest: each with the structural UNSAT argument tools/unsat_proofs.py
    finds (unit propagation, an empty interval, a folded `x <u 0`), or "open"
    (argued per family in DESIGN.md).  The arguments are re-derived here."""
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))
    import unsat_proofs
    from mythril_amd.compiler import _flatten
    gt = _ground_truth()
    reasons = {}
    for f, why in gt["no_witness"].items():
        reasons[why["reason"]] = reasons.get(why["reason"], 0) + 1
        if why["reason"] == "open":
            continue
        s = parse_file(os.path.join(CORPUS, f))
        if why["reason"] in ("rewriting", "contradiction", "bounds"):
            got = unsat_proofs.abstract(s.asserts, s.ctx)     # on the query as stated (round 6)
        else:
            q = prepare(s.asserts, s.ctx)
            conj = _flatten(q.lowered.conjuncts)
            got = {"propagation": unsat_proofs.propagation, "interval": unsat_proofs.interval,
                   "tautology": lambda c: unsat_proofs.tautology(c, q.ctx)}[why["reason"]](conj)
        assert got is not None and got["reason"] == why["reason"], f
    # at most 8 queries without a witness or a reason
    assert reasons.get("open", 0) <= 8 and sum(reasons.values()) == len(gt["no_witness"])


def test_unsat_arguments_never_fire_on_satisfiable_queries():
    """Soundness check of tools/unsat_proofs.py's rewriting / contradiction /
    bounds arguments: on every query the device witnessed (each witness holds
    under the oracle, test_ground_truth_witnesses_hold) and every followed
    successor (satisfied by the concolic model), none of them claims UNSAT."""
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))
    import unsat_proofs
    gt = _ground_truth()
    checked = 0
    for m in MANIFEST:
        if m["file"] in gt["no_witness"]:
            continue
        s = parse_file(os.path.join(CORPUS, m["file"]))
        assert unsat_proofs.abstract(s.asserts, s.ctx) is None, m["file"]
        checked += 1
    assert checked >= 760
