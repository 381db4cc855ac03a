"""Replay of concolic LASER runs through the real plugin hooks, in LaserEVM's
order (TEST INFRASTRUCTURE).

``tests/laser_concolic.py`` records, per transaction, every JUMPI's successor
constraint sets and every concrete SHA3 of the path it follows over the
reference's bytecode.  This module plays those events into
``mythril_amd.mythril_plugin.WitnessBatchingLaserPlugin`` through a stand-in
LaserEVM that fires them in the order of ``mythril/laser/ethereum/svm.py``:

* transaction i > 1 starts with the reachability prune of the open states
  (``svm.py:216-223``: ``state.constraints.is_possible`` for each), after the
  previous transaction's ``stop_sym_trans`` hooks (``svm.py:244-245``);
* inside a transaction, each JUMPI's successors pass through the post hooks
  (``svm.py:_execute_post_hook``, ``:694-697``) and are then pruned one by one
  with ``is_possible`` (``svm.py:287-292``);
* each concrete SHA3 asks ``find_concrete_keccak``
  (``keccak_function_manager.py:57-69``), here the installed Keccak service;
* ``stop_sym_exec`` hooks at the end (``svm.py:205-206``).

The constraint sets are ``Constraints`` objects (a list subclass with
``get_all_constraints()``, ``state/constraints.py:10-108``), never tuples, so
the drop-in's non-tuple path (``model.py`` ``get_all_constraints``) is the one
exercised.  The open state carried across a transaction boundary is the
followed successor of the transaction's last JUMPI (the concolic path), when
the transaction did not revert.
"""
from __future__ import annotations

import sys
import types
from functools import lru_cache
from typing import Dict, List

from oracle.dag_eval import ArrayVal, eval_nodes
from oracle.keccak import keccak256
from tests.laser_concolic import ACTORS, run_sequence


class UnsatError(Exception):
    pass


class FakeRaw:
    def __init__(self, node):
        self.node = node

    def get_id(self):
        return self.node.id

    def eq(self, other):
        return isinstance(other, FakeRaw) and other.node is self.node


class FakeBool:
    def __init__(self, node):
        self.raw = FakeRaw(node)

    def __hash__(self):
        return self.raw.node.id

    def __eq__(self, other):
        return isinstance(other, FakeBool) and other.raw.node.id == self.raw.node.id


class Model:
    def __init__(self, raw):
        self.raw = raw


class Constraints(list):
    """state/constraints.py:10-108: a list of Bools; ``is_possible`` calls the
    get_model bound in the constraints module; ``get_all_constraints`` adds the
    keccak conditions (here the last element of a recorded set, when present)."""

    def __init__(self, items, keccak_cond=None):
        super().__init__(items)
        self.keccak_cond = keccak_cond

    @property
    def is_possible(self) -> bool:
        gm = sys.modules["mythril.laser.ethereum.state.constraints"].get_model
        try:
            gm(self)
        except UnsatError:
            return False
        return True

    def get_all_constraints(self):
        return self[:] + ([self.keccak_cond] if self.keccak_cond is not None else [])

    def __hash__(self):
        return tuple(self[:]).__hash__()


class ReplayVM:
    """Stand-in LaserEVM: hook registry + the event order of svm.py."""

    def __init__(self):
        self.laser_hooks: Dict[str, list] = {}
        self.post_hooks: Dict[str, list] = {}
        self.open_states: list = []
        self.counts = {"is_possible": 0, "tx_prunes": 0, "jumpi_prunes": 0, "keccaks": 0, "module_queries": 0,
                       "tuple_queries": 0}

    def register_laser_hooks(self, kind, hook):
        self.laser_hooks.setdefault(kind, []).append(hook)

    def register_hooks(self, kind, hooks):
        assert kind == "post"
        for op, fs in hooks.items():
            self.post_hooks.setdefault(op, []).extend(fs)

    def _fire(self, kind):
        for h in self.laser_hooks.get(kind, []):
            h()

    def _possible(self, cons: Constraints) -> bool:
        self.counts["is_possible"] += 1
        return cons.is_possible

    def _module(self, cons: Constraints) -> bool:
        solver = sys.modules["mythril.analysis.solver"]
        try:
            solver.get_model(cons)
            return True
        except UnsatError:
            return False

    def replay(self, runs, keccak=None) -> List[bool]:
        """Play every run (one concolic transaction sequence each) in LASER's
        order; returns the is_possible answers of the JUMPI successors."""
        answers = []
        for run, n_tx in runs:
            self.open_states = []
            kk = list(run.keccaks)
            for tx in range(1, n_tx + 1):
                if tx > 1:
                    self._fire("stop_sym_trans")      # end of the previous transaction
                    kept = []
                    for ws in self.open_states:        # svm.py:216-223 (open states are WorldStates)
                        self.counts["tx_prunes"] += 1
                        if self._possible(ws.constraints):
                            kept.append(ws)
                    self.open_states = kept
                last_followed = None
                qs = [(i, q) for i, q in enumerate(run.queries) if q.tx == tx]
                j = 0
                while j < len(qs):
                    if qs[j][1].kind != "jumpi":
                        # a detection module's own query: analysis.solver.get_model
                        # on the state's Constraints plus its conditions
                        while kk and kk[0][0] == tx and kk[0][1] <= qs[j][0]:
                            self._keccak(keccak, kk.pop(0))
                        self.counts["module_queries"] += 1
                        q = qs[j][1]
                        if q.tuple_form:
                            # DependencyPruner's get_model((location == dependency,)): a
                            # tuple, so the drop-in adds no keccak conditions (model.py:35-36)
                            self.counts["tuple_queries"] += 1
                            answers.append(self._module(tuple(FakeBool(n) for n in q.constraints)))
                        else:
                            answers.append(self._module(_state(q).world_state.constraints))
                        j += 1
                        continue
                    # one JUMPI: its successor sets are recorded consecutively
                    grp = [qs[j]]
                    while j + len(grp) < len(qs) and qs[j + len(grp)][1].pc == qs[j][1].pc and len(grp) < 2 \
                            and qs[j + len(grp)][1].kind == "jumpi":
                        grp.append(qs[j + len(grp)])
                    # concrete SHA3s executed before this JUMPI
                    while kk and kk[0][0] == tx and kk[0][1] <= grp[0][0]:
                        self._keccak(keccak, kk.pop(0))
                    states = [_state(q) for _, q in grp]
                    for st in states:                  # svm.py:694-697 post hooks
                        for h in self.post_hooks.get("JUMPI", []):
                            h(st)
                    for (_, q), st in zip(grp, states):  # svm.py:287-292
                        self.counts["jumpi_prunes"] += 1
                        ok = self._possible(st.world_state.constraints)
                        answers.append(ok)
                        if q.taken:
                            last_followed = st
                    j += len(grp)
                while kk and kk[0][0] == tx:
                    self._keccak(keccak, kk.pop(0))
                if run.halts[tx - 1] in ("STOP", "RETURN", "SELFDESTRUCT") and last_followed is not None:
                    self.open_states = [last_followed.world_state]
            self._fire("stop_sym_trans")
        self._fire("stop_sym_exec")
        return answers

    def _keccak(self, keccak, ev):
        _, _, bits, value = ev
        self.counts["keccaks"] += 1
        if keccak is not None:
            got = keccak(value, bits)
            assert got == int.from_bytes(keccak256(value.to_bytes(bits // 8, "big")), "big")


def _state(q):
    cons = list(q.constraints)
    kc = None
    if q.keccak_cond is not None:     # get_all_constraints() adds it back
        assert cons[-1] is q.keccak_cond
        kc = FakeBool(cons.pop())
    c = Constraints([FakeBool(n) for n in cons], kc)
    # a LASER world state holds the target contract's account (its address is
    # a storage key the plugin's Keccak speculation hashes, mythril_plugin.storage_keys)
    from tests.laser_concolic import CONTRACT
    return types.SimpleNamespace(world_state=types.SimpleNamespace(constraints=c, accounts={CONTRACT: None}))


def install_standins(monkeypatch, model_for, ctx):
    """Stand-in Mythril modules (as tests/test_dropin.py) whose reference
    get_model answers from ``model_for(nodes)``: a model dict (SAT) or None
    (UnsatError)."""
    from mythril_amd import z3bridge
    from mythril_amd.smt2 import Script
    calls = {"reference": 0}
    args = types.SimpleNamespace(solver_timeout=10000, solver_log=None)
    th = types.SimpleNamespace(time_remaining=lambda: 10 ** 9)

    @lru_cache(maxsize=2 ** 23)
    def reference_get_model(constraints, minimize=(), maximize=(), enforce_execution_time=True):
        calls["reference"] += 1
        cl = constraints if type(constraints) == tuple else constraints.get_all_constraints()
        m = model_for([c.raw.node for c in cl if type(c) != bool])
        if m is None:
            raise UnsatError
        return Model(["ref", m])

    mods = {
        "mythril": types.ModuleType("mythril"),
        "mythril.exceptions": types.SimpleNamespace(UnsatError=UnsatError),
        "mythril.support": types.ModuleType("mythril.support"),
        "mythril.support.support_args": types.SimpleNamespace(args=args),
        "mythril.support.model": types.SimpleNamespace(get_model=reference_get_model),
        "mythril.laser": types.ModuleType("mythril.laser"),
        "mythril.laser.ethereum": types.ModuleType("mythril.laser.ethereum"),
        "mythril.laser.ethereum.time_handler": types.SimpleNamespace(time_handler=th),
        "mythril.laser.ethereum.state": types.ModuleType("mythril.laser.ethereum.state"),
        "mythril.laser.ethereum.state.constraints": types.SimpleNamespace(get_model=reference_get_model),
        "mythril.analysis": types.ModuleType("mythril.analysis"),
        "mythril.analysis.solver": types.SimpleNamespace(get_model=reference_get_model),
        "mythril.laser.smt": types.ModuleType("mythril.laser.smt"),
        "mythril.laser.smt.model": types.SimpleNamespace(Model=Model),
    }
    for k, v in mods.items():
        monkeypatch.setitem(sys.modules, k, v)
    mods["mythril"].support = mods["mythril.support"]
    mods["mythril"].analysis = mods["mythril.analysis"]
    mods["mythril"].laser = mods["mythril.laser"]
    mods["mythril.support"].model = mods["mythril.support.model"]
    mods["mythril.analysis"].solver = mods["mythril.analysis.solver"]
    mods["mythril.laser"].ethereum = mods["mythril.laser.ethereum"]
    mods["mythril.laser.ethereum"].state = mods["mythril.laser.ethereum.state"]
    mods["mythril.laser.ethereum.state"].constraints = mods["mythril.laser.ethereum.state.constraints"]

    def to_ir(raws, c=None):
        s = Script(ctx)
        s.asserts = [r.node for r in raws]
        return s

    def confirm(raws, script, w, timeout_ms=2000):
        """The "z3 re-check": the oracle evaluates the ORIGINAL formula under
        the witness (arrays and UF tables included)."""
        model = dict(w.values)
        for n, cells in w.arrays.items():
            model[n] = ArrayVal(cells)
        for n, table in w.functions.items():
            model[n] = (dict(table), 0)
        vals = eval_nodes([r.node for r in raws], model)
        return ("z3", model) if all(vals[r.node.id] for r in raws) else None

    monkeypatch.setattr(z3bridge, "to_ir", to_ir)
    monkeypatch.setattr(z3bridge, "model_from_witness", confirm)
    return calls


def concolic_runs(contracts=None):
    """[(ConcolicLaser, Run, n_tx)] for the corpus scenarios (tools/make_laser_corpus.py)."""
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    from make_laser_corpus import SCENARIOS, load_code, scenario_balances
    out = []
    for contract, scenarios in SCENARIOS.items():
        if contracts and contract not in contracts:
            continue
        code = load_code(contract)
        for name, txs, *opt in scenarios:
            opts = opt[0] if opt else {}
            m, run = run_sequence(code, txs, storage=opts.get("storage"), balances=scenario_balances(opts))
            out.append((f"{contract}/{name}", m, run, len(txs)))
    return out
