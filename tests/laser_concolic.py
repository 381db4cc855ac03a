"""Concolic restatement of LASER's path constraints over reference-held bytecode
(TEST INFRASTRUCTURE: generates fixtures; never imported by mythril_amd/).

The reference ships runtime bytecode that needs no solc
(``/root/reference/tests/testdata/inputs/*.sol.o``; e.g. ``underflow.sol.o``
is ``solidity_examples/token.sol`` with ``transfer`` renamed ``sendeth``,
``suicide.sol.o`` is config C1's contract).  This module executes such code
the way LASER does, with symbolic inputs, while following ONE concrete path
chosen by a concrete input model (concolic execution), and records the
constraint set LASER would hold at every JUMPI:

* free variables with LASER's names: ``{tx}_calldata`` (Array 256->8) and
  ``{tx}_calldatasize`` (``state/calldata.py:214-215``), ``sender_{tx}``,
  ``call_value{tx}``, ``gas_price{tx}`` (``transaction/symbolic.py:118-136``),
  the ``balance`` array (``state/world_state.py:33``) and the account's
  symbolic ``Storage`` array (``state/account.py:26-29``);
* per transaction: ``Or(sender == actor for the 3 ACTORS)``
  (``transaction/symbolic.py:210-212``), ``UGE(balance[sender], value)`` and the
  balance transfer (``transaction/transaction_models.py:139-143``);
* calldata reads ``If(i <s size, calldata[i], 0)`` (``calldata.py:218-231``,
  signed ``<`` of ``smt/bitvec.py:138-180``), words as ``Concat`` of 32 reads;
* opcode terms as ``laser/ethereum/instructions.py`` builds them (comparisons
  are Bools, ``util.pop_bitvec`` turns a Bool into ``If(b, 1, 0)``, ISZERO of a
  Bool is ``Not``, EQ wraps Bool operands), with z3-``simplify``-like folding of
  constant subterms and of byte-wise memory round trips;
* JUMPI (``instructions.py:1556-1633``): the taken successor appends ``cond``
  (a Bool) or ``cond != 0``; the other ``Not(cond)`` / ``cond == 0``.  LASER
  prunes each successor with ``is_possible`` (``svm.py:287-292``), so both
  successor sets are feasibility queries;
* keccak of symbolic memory is the UF ``keccak256_N`` with the manager's
  conditions appended by ``get_all_constraints`` (tests/mythril_shapes.py);
* contract creation (``transaction_models.py:195-260``): the init code runs
  with a concrete CREATOR, storage ``K(256, 256, 0)`` (``account.py:26-29``),
  the new account's balance set to 0 (``world_state.py:145-166``); its RETURN
  data becomes the runtime code of the later message calls;
* the environment leaves of ``global_state.py:126-136`` /
  ``environment.py:47-48``: ``{tx}_timestamp``, ``block_number``,
  ``{tx}_coinbase``, ``{tx}_block_difficulty``, ``chain_id``, ``{tx}_gas``,
  ``{tx}_returndatasize``; ORIGIN is the transaction's ``sender_{tx}``;
* EXP through the ``Power`` UF with the exponent manager's conditions
  (``exponent_function_manager.py:21-58``, ``instructions.py:623-636``);
* CALL / CALLCODE / DELEGATECALL / STATICCALL to a symbolic callee: an ether
  transfer (``instructions.py:1960-2000``, ``transfer_ether :72-93``) and a
  fresh ``{tx}_retval_{pc}``;
* the detection modules' own ``get_model`` queries (``Query.kind``):
  EtherThief's balance increase after CALL/STATICCALL (``ether_thief.py:60-76``),
  StateChangeAfterCall's external-call and balance-change checks
  (``state_change_external_calls.py:119-140,183-197``), and the integer
  module's overflow checks at the end of a transaction (``integer.py:140-160,
  245-277``, annotations propagated as ``smt/bitvec.py`` unions them).

The concrete model satisfies every constraint set on the path it follows
(checked with the oracle when the corpus is made), so the taken-branch
queries are SAT with a known witness; the other successors' status is
unknown without a solver.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from mythril_amd.ir import BOOL, Ctx, Node
from oracle import bvsem as S
from oracle.dag_eval import ArrayVal, _eval1, eval_nodes
from oracle.keccak import keccak256
from tests.mythril_shapes import PART, KeccakManager

M256 = (1 << 256) - 1
ACTORS = {"CREATOR": 0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE,
          "ATTACKER": 0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF,
          "SOMEGUY": 0xAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAA}
CONTRACT = 0x0901D12EBE1B195E5AA8748E62BD7734AE19B51F   # LASER's default target address


class Halt(Exception):
    pass


class Unsupported(Exception):
    pass


@dataclass
class TxInput:
    """One message call's concrete choice (the path the concolic run follows)."""
    calldata: bytes
    sender: int = ACTORS["ATTACKER"]
    value: int = 0
    gas_price: int = 1
    retvals: Dict[int, int] = field(default_factory=dict)   # CALL pc (-1: any) -> {tx}_retval_{pc} (default 1)
    env: Dict[str, int] = field(default_factory=dict)       # timestamp, block_number, gas, ... (model values)
    creation: bool = False                                  # contract creation: the code is init code


@dataclass
class Query:
    """A feasibility query LASER would send to get_model at a JUMPI successor."""
    tx: int
    pc: int
    taken: bool                    # the successor the concrete path follows
    constraints: List[Node]        # world-state constraints + keccak conditions
    sat: Optional[bool]            # True for the followed successor; None = unknown
    keccak_cond: Optional[Node] = None   # the manager's conditions: the last element of constraints
    kind: str = "jumpi"            # "jumpi", or the detection module / plugin whose get_model asks it
    tuple_form: bool = False       # get_model((...,)): a tuple, so no keccak conditions (model.py:35-36)


@dataclass
class Run:
    queries: List[Query] = field(default_factory=list)
    model: Dict = field(default_factory=dict)
    halts: List[str] = field(default_factory=list)
    keccaks: List[Tuple[int, int, int, int]] = field(default_factory=list)   # (tx, queries so far, bits, value)


class ConcolicLaser:
    def __init__(self, code: bytes, storage: Optional[Dict[int, int]] = None, balances: Optional[Dict[int, int]] = None):
        self.c = Ctx()
        self.code = code
        self.jumpdests = self._jumpdests(code)
        self.km = KeccakManager(self.c)
        self.keccak_index: Dict[Tuple[int, int], int] = {}   # (width, input) -> k: UF value lower + 64 k
        self.constraints: List[Node] = []
        stor_name = f"Storage[{CONTRACT}]"
        self.storage = self.c.array(stor_name, 256, 256)
        self.balance = self.c.array("balance", 256, 256)
        self.balance0 = self.balance               # world_state.starting_balances (world_state.py:33-34)
        self.model: Dict = {stor_name: ArrayVal(dict(storage or {}), 0),
                            "balance": ArrayVal(dict(balances or {}), 0),
                            "Power": ({}, 0)}
        self.vals: Dict[int, object] = {}
        self.run_log = Run()
        # analysis/symbolic.py:100-117: the actor accounts in the world state
        # (CREATOR only when there is creation code), then the contract
        self.accounts: List[int] = [ACTORS["ATTACKER"], CONTRACT]
        self.power_sent = False                    # exponent_function_manager.concrete_constraints_sent
        # integer module (integer.py): node id -> annotation indices, and the
        # annotations (kind, tx, pc, constraints at the operation, overflow condition)
        self.ann: Dict[int, frozenset] = {}
        self.annotations: List[Tuple[str, int, int, List[Node], Node]] = []
        self.tx_anns: set = set()
        self.tx = 0
        # PredictableVars (dependence_on_predictable_vars.py): node id -> the
        # PredictableValueAnnotation operations it carries
        self.pred: Dict[int, frozenset] = {}
        self.deps = DependencyPruner()
        self.mutated = False                        # MutationPruner's MutationAnnotation (this tx)
        self.creation_txs: set = set()
        self.deleted = False                        # SELFDESTRUCT ran: later message calls are skipped
        self.sequence: List[int] = []               # world_state.transaction_sequence: the txs that ended without revert

    # ---------------------------------------------------------------- terms
    @staticmethod
    def _jumpdests(code):
        """JUMPDEST offsets.  ``code`` is bytes, or a list of ints and 8-bit
        terms: runtime code returned by a constructor that patched symbolic
        immutables into it (transaction_models.py:252-262 assign_bytecode of
        the RETURN data; disassembler/asm.py:120-140 keeps symbolic PUSH
        arguments).  A symbolic byte is never an opcode here (it sits inside
        PUSH data)."""
        out, i = set(), 0
        while i < len(code):
            op = code[i]
            if not isinstance(op, int):
                i += 1
                continue
            if op == 0x5B:
                out.add(i)
            i += (op - 0x5F + 1) if 0x60 <= op <= 0x7F else 1
        return out

    def k(self, v: int, w: int = 256) -> Node:
        return self.c.const(v, w)

    def val(self, n: Node):
        """Concrete value of a term under the model (what the followed path sees)."""
        got = self.vals.get(n.id)
        if got is None:
            for m in _postorder(n, self.vals):
                self.vals[m.id] = self._eval(m)
            got = self.vals[n.id]
        return got

    def _eval(self, m: Node):
        if m.op == "apply":
            d, default = self.model.get(m.name, ({}, 0))
            return d.get(tuple(self.vals[a.id] for a in m.args), default) & ((1 << m.width) - 1)
        return _eval1(m, [self.vals[a.id] for a in m.args], self.model)

    def app(self, op: str, *args: Node, params=()) -> Node:
        """Build a term, folding what z3's simplify folds (constant operands, the
        concat of a term's own byte slices, select over a store chain with
        constant keys, x+0, x>=u 0, x=x), and carrying the integer module's
        annotations from the operands to the result as smt/bitvec.py does
        (not through array reads: BaseArray.__getitem__ starts a fresh BitVec)."""
        r = self._app(op, *args, params=params)
        for tags in (self.ann, self.pred):
            if tags and op not in ("select", "store", "apply"):
                u = frozenset().union(*[tags.get(a.id, frozenset()) for a in args])
                if u:
                    tags[r.id] = tags.get(r.id, frozenset()) | u
        return r

    def _app(self, op: str, *args: Node, params=()) -> Node:
        c = self.c
        if op == "concat":
            args = _merge_slices(c, list(args))
            if len(args) == 1:
                return args[0]
        if args and all(a.op == "const" for a in args) and op not in ("select", "store"):
            t = c.app(op, *args, params=params)
            v = _eval1(t, [a.val for a in args], {})
            return c.const(v, t.width)
        if op == "select":
            arr, key = args
            while arr.op == "store" and key.op == "const" and arr.args[1].op == "const":
                if arr.args[1].val == key.val:
                    return arr.args[2]
                arr = arr.args[0]
            if arr.op == "const_array":
                return arr.args[0]
            return c.app("select", arr, key)
        if op == "store" and args[0].op == "store" and args[1].op == "const" and args[0].args[1] is args[1]:
            return c.app("store", args[0].args[0], args[1], args[2])     # store(store(a,k,_),k,v)
        if op in ("bvadd", "bvsub") and args[1].op == "const" and args[1].val == 0:
            return args[0]
        if op == "bvadd" and args[0].op == "const" and args[0].val == 0:
            return args[1]
        if op == "bvuge" and args[1].op == "const" and args[1].val == 0:
            return c.true()
        if op == "=" and args[0] is args[1]:
            return c.true()
        if op == "extract" and args[0].op == "concat":
            # slice of a concat that falls inside one operand
            hi, lo = params
            off = args[0].width
            for a in args[0].args:
                off -= a.width
                if lo >= off and hi < off + a.width:
                    return self.app("extract", a, params=(hi - off, lo - off)) if a.width != hi - lo + 1 else a
        if op == "extract" and params[0] == args[0].width - 1 and params[1] == 0:
            return args[0]
        if op == "bvand" and len(args) == 2:   # and(m, and(m, x)) = and(m, x)
            x, y = args
            for p, q in ((x, y), (y, x)):
                if p.op == "const" and q.op == "bvand" and any(t is p for t in q.args):
                    return q
        return c.app(op, *args, params=params)

    def bv(self, x: Node) -> Node:
        """util.pop_bitvec: a Bool on the stack becomes If(b, 1, 0)."""
        if x.width == BOOL:
            if x.op == "const":
                return self.k(x.val)
            return self.app("ite", x, self.k(1), self.k(0))
        return x

    def leaf(self, name: str, value: int, w: int = 256) -> Node:
        self.model.setdefault(name, value)
        return self.c.var(name, w)

    # ---------------------------------------------------------------- keccak
    def sha3(self, data: Node) -> Node:
        """keccak_function_manager.create_keccak: concrete data -> the real hash;
        symbolic -> keccak256_N(data), whose model value is the manager's
        interval value (lower + 64 k, distinct per input) so that the model also
        satisfies create_conditions."""
        if data.op == "const":
            # LASER hashes concrete data on the spot (find_concrete_keccak): logged
            # with its position among the queries for tests/laser_replay.py
            self.run_log.keccaks.append((self.tx, len(self.run_log.queries), data.width, data.val))
            h = self.km.create_keccak(data)
            # the manager's concrete-hash conditions (keccak256_N(data) == h, and the
            # inverse) hold in the model too
            n = data.width
            self.model.setdefault(f"keccak256_{n}", ({}, 0))[0][(data.val,)] = h.val
            self.model.setdefault(f"keccak256_{n}-1", ({}, 0))[0][(h.val,)] = data.val
            return h
        n = data.width
        fx = self.km.create_keccak(data)
        x = self.val(data)
        key = (n, x)
        if key not in self.keccak_index:
            self.keccak_index[key] = len([1 for kk in self.keccak_index if kk[0] == n])
        self.km._create_condition(data)   # fixes the width's interval hook in creation order
        lower = self.km.interval_hook_for_size[n] * PART
        y = (lower + 63) // 64 * 64 + 64 * self.keccak_index[key]   # in the interval, 64-aligned
        fwd = self.model.setdefault(f"keccak256_{n}", ({}, 0))[0]
        inv = self.model.setdefault(f"keccak256_{n}-1", ({}, 0))[0]
        fwd[(x,)] = y
        inv[(y,)] = x
        self.vals.pop(fx.id, None)
        return fx

    # ---------------------------------------------------------------- EXP
    def power(self, b: Node, e: Node) -> Node:
        """exponent_function_manager.create_condition (``:34-58``): the result is
        the UF application Power(b, e); the condition goes to the world state."""
        c = self.c
        fx = c.apply("Power", 256, b, e)
        tab = self.model["Power"][0]
        bv, ev = self.val(b), self.val(e)
        if b.op == "const" and e.op == "const":
            v = pow(b.val, e.val, 1 << 256)
            tab[(bv, ev)] = v
            self.vals.pop(fx.id, None)
            self.constraints.append(self.app("=", self.k(v), fx))
            return self.k(v)
        conds = [self.app("bvsgt", fx, self.k(0))]
        if not self.power_sent:
            for i in range(32):
                conds.append(self.app("=", c.apply("Power", 256, self.k(256), self.k(i)), self.k(256 ** i)))
                tab[(256, i)] = 256 ** i
            self.power_sent = True
        if b.op == "const" and b.val == 256:
            conds.append(self.app("=", c.apply("Power", 256, b, self.app("bvurem", e, self.k(32))), fx))
            tab[(256, ev % 32)] = 256 ** (ev % 32)
            tab[(bv, ev)] = 256 ** (ev % 32)          # the UF the conditions pin down
        else:
            tab[(bv, ev)] = pow(bv, ev, 1 << 256)
        self.vals.clear()
        self.constraints.append(conds[0] if len(conds) == 1 else self.app("and", *conds))
        return fx

    # ---------------------------------------------------------------- queries
    def query_set(self, extra=()) -> List[Node]:
        """Constraints.get_all_constraints(): the world constraints (+ a module's
        extra conjuncts) + keccak conditions."""
        cond = self.km.create_conditions()
        tail = [] if (cond.op == "const" and cond.val) else [cond]
        body = [x for x in list(self.constraints) + list(extra) if not (x.op == "const" and x.val)]
        return body + tail

    def module_query(self, kind: str, extra, base: Optional[List[Node]] = None, first: bool = False) -> Optional[bool]:
        """A detection module's get_model(constraints + extra) (``first``:
        ``Constraints(extra) + constraints``, the extra conjuncts leading):
        recorded with status sat when the concrete model satisfies it, else
        unknown.  Returns that status (None: folded to False, not asked)."""
        saved = self.constraints
        if base is not None:
            self.constraints = base
        try:
            extra = [self.bv(x) if x.width != BOOL else x for x in extra]
            if first:
                cond = self.km.create_conditions()
                qset = [x for x in list(extra) + list(self.constraints) if not (x.op == "const" and x.val)] + \
                    ([] if (cond.op == "const" and cond.val) else [cond])
            else:
                qset = self.query_set(extra)
        finally:
            self.constraints = saved
        if any(x.op == "const" and not x.val for x in qset):
            return None               # folded to False: nothing to ask
        kc = qset[-1] if self.km.create_conditions().op != "const" else None
        ok = check_model(qset, self.model)
        self.run_log.queries.append(Query(self.tx, self.pc, True, qset, True if ok else None, kc, kind))
        return bool(ok)

    def tuple_query(self, kind: str, conds: List[Node]) -> Optional[bool]:
        """get_model((c, ...)) with a tuple (dependency_pruner.py:164,180,190):
        no keccak conditions are added (model.py:35-36).  Constant answers are
        not asked of the engine (z3 folds them); returns True/False for them,
        else the recorded status (True: the model satisfies it; None: unknown)."""
        if all(x.op == "const" for x in conds):
            return all(x.val for x in conds)
        ok = check_model(conds, self.model)
        self.run_log.queries.append(Query(self.tx, self.pc, True, list(conds), True if ok else None, None, kind,
                                          tuple_form=True))
        return True if ok else None

    def annotate(self, kind: str, op0: Node, res: Node, cond: Node) -> None:
        """integer.py:_handle_add/_mul/_sub: the overflow condition annotates
        the first operand (a constant operand: the result)."""
        if cond.op == "const":
            return
        idx = len(self.annotations)
        self.annotations.append((kind, self.tx, self.pc, list(self.constraints), cond))
        tgt = op0 if op0.op != "const" else res
        self.ann[tgt.id] = self.ann.get(tgt.id, frozenset()) | {idx}
        if tgt is not res:
            self.ann[res.id] = self.ann.get(res.id, frozenset()) | {idx}

    def collect(self, x: Node) -> None:
        """integer.py:_handle_sstore/_jumpi/_call/_return: annotations reaching a sink."""
        self.tx_anns |= self.ann.get(x.id, frozenset())

    def tx_end_queries(self) -> None:
        """integer.py:_handle_transaction_end (``:245-277``): for each collected
        annotation, get_model(ostate constraints + [condition])."""
        for idx in sorted(self.tx_anns):
            kind, _, _, ostate, cond = self.annotations[idx]
            self.module_query(f"IntegerArithmetics/{kind}", [cond], base=ostate)
        self.tx_anns = set()

    # ---------------------------------------------------------------- transactions
    def _setup_tx(self, tx: int, inp: TxInput, sender: Node, me: Node) -> None:
        c = self.c
        value = self.leaf(f"call_value{tx}", inp.value)
        self.leaf(f"gas_price{tx}", inp.gas_price)
        size = self.leaf(f"{tx}_calldatasize", len(inp.calldata))
        self.model[f"{tx}_calldata"] = ArrayVal(dict(enumerate(inp.calldata)), 0)
        for name, v in inp.env.items():
            self.model[name if name in ("block_number", "chain_id") else f"{tx}_{name}"] = v
        self.cd = c.array(f"{tx}_calldata", 256, 8)
        self.cdsize = size
        self.sender, self.value, self.tx, self.inp = sender, value, tx, inp
        self.returndata = None
        self.tx_anns = set()
        # transaction_models.py:139-143 then transaction/symbolic.py:210-212
        self.constraints.append(self.app("bvuge", self.app("select", self.balance, sender), value))
        self.balance = self.app("store", self.balance, me, self.app("bvadd", self.app("select", self.balance, me), value))
        self.balance = self.app("store", self.balance, sender,
                                self.app("bvsub", self.app("select", self.balance, sender), value))
        orc = c.app("or", *[self.app("=", sender, self.k(a)) for a in ACTORS.values()]) \
            if sender.op != "const" else c.true()
        if not (orc.op == "const" and orc.val):
            self.constraints.append(orc)
        self.vals.clear()

    def message_call(self, tx: int, inp: TxInput, max_steps: int = 20000) -> str:
        sender = self.leaf(f"sender_{tx}", inp.sender)
        self.deps.iteration += 1        # start_sym_trans (svm.py:239-240; dependency_pruner.py:204-206)
        self._setup_tx(tx, inp, sender, self.k(CONTRACT))
        self.mutated = False
        res = self._exec(max_steps)
        if res in ("STOP", "RETURN", "SELFDESTRUCT"):
            self.end_world_state(False)
        return res

    def contract_creation(self, tx: int, inp: TxInput, max_steps: int = 20000) -> str:
        """ContractCreationTransaction (transaction_models.py:195-245): CREATOR
        calls the init code; the new account has concrete storage K(256,256,0)
        and balance 0; the RETURN data becomes the runtime code."""
        if ACTORS["CREATOR"] not in self.accounts:
            self.accounts.insert(0, ACTORS["CREATOR"])
        self.storage = self.c.const_array(256, self.k(0))
        self.balance = self.app("store", self.balance, self.k(CONTRACT), self.k(0))
        self.creation_txs.add(tx)
        self._setup_tx(tx, inp, self.k(inp.sender), self.k(CONTRACT))
        self.mutated = False
        res = self._exec(max_steps)
        if res == "RETURN":
            self.code = self.returned
            self.jumpdests = self._jumpdests(self.code)
            if len(self.code):        # transaction_models.py:252-262 / svm.py:416-425
                self.end_world_state(True)
        return res

    def _calldata_byte(self, i: Node) -> Node:
        return self.app("ite", self.app("bvslt", i, self.cdsize), self.app("select", self.cd, i), self.k(0, 8))

    def _env_leaf(self, name: str, default: int) -> Node:
        """global_state.new_bitvec (global_state.py:126-136): '{tx}_{name}'."""
        full = f"{self.tx}_{name}"
        return self.leaf(full, self.model.get(full, default))

    def _transfer(self, sender: Node, receiver: Node, value: Node) -> None:
        """instructions.py:72-93 transfer_ether."""
        self.constraints.append(self.app("bvuge", self.app("select", self.balance, sender), value))
        self.balance = self.app("store", self.balance, receiver,
                                self.app("bvadd", self.app("select", self.balance, receiver), value))
        self.balance = self.app("store", self.balance, sender,
                                self.app("bvsub", self.app("select", self.balance, sender), value))
        self.vals.clear()

    def _predictable(self, op: str, x: Node) -> Node:
        """PredictableVars post hook of COINBASE / TIMESTAMP / NUMBER
        (dependence_on_predictable_vars.py:176-184): the pushed value carries a
        PredictableValueAnnotation (GASLIMIT is a constant here; not tagged)."""
        self.pred[x.id] = self.pred.get(x.id, frozenset()) | {op}
        return x

    def _blockhash(self, param: Node) -> Node:
        """PredictableVars BLOCKHASH pre hook (dependence_on_predictable_vars.py:
        142-159): get_model(world constraints + [ULT(param, block_number),
        ULT(block_number, 2^255)]); if SAT the state gets an
        OldBlockNumberUsedAnnotation and the post hook tags the hash.  The hash
        is the fresh symbol '{tx}_blockhash_block_{param}' (instructions.py:
        1369-1380)."""
        param = self.bv(param)
        bn = self.leaf("block_number", 10_000_000)
        ok = self.module_query("PredictableVars/blockhash",
                               [self.c.app("bvult", param, bn), self.c.app("bvult", bn, self.k(1 << 255))])
        h = self._env_leaf(f"blockhash_block_{_z3_str(param)}", 0x1234)
        if ok:
            self.pred[h.id] = self.pred.get(h.id, frozenset()) | {"blockhash"}
        return h

    @staticmethod
    def _assertion_failure(off: Node, ln: Node, mbyte) -> bool:
        """exceptions.py is_assertion_failure: concrete offset and length, the
        data starts with Panic(uint256)'s selector 4e487b71 and ends in 0x01."""
        if off.width == BOOL or ln.width == BOOL or off.op != "const" or ln.op != "const" or ln.val < 5:
            return False
        data = [mbyte(off.val + i) for i in range(ln.val)]
        if not all(x.op == "const" for x in data[:4] + data[-1:]):
            return False
        return [x.val for x in data[:4]] == [78, 72, 123, 113] and data[-1].val == 1

    def _selfdestruct(self, to: Node) -> None:
        """AccidentallyKillable SELFDESTRUCT pre hook (suicide.py:50-96): for every
        message call of the sequence And(caller == ATTACKER, caller == origin)
        (caller and origin are the one 'sender_N' symbol); get_transaction_
        sequence(world + [to == ATTACKER] + those), and without a model of that,
        world + those alone."""
        c = self.c
        att = self.k(ACTORS["ATTACKER"])
        ac = []
        for t in self.sequence + [self.tx]:
            if t in self.creation_txs:
                continue
            s = c.var(f"sender_{t}", 256)
            ac.append(c.app("and", c.app("=", s, att), c.app("=", s, s)))
        ok = self.module_query("AccidentallyKillable/attacker_beneficiary", [self.app("=", to, att)] + ac)
        if not ok:
            self.module_query("AccidentallyKillable/any_sender", ac)
        self.deleted = True

    def end_world_state(self, creation: bool) -> None:
        """svm.py:416-425: a transaction that ends without revert adds its
        world state; the add_world_state hooks run.  MutationPruner
        (mutation_pruner.py:60-86): for a message call, get_model(world
        constraints + [UGT(callvalue, 0)]) (a Constraints: keccak conditions
        included); UNSAT with no mutation on the path drops the world state
        (the scenarios put non-mutating calls last).  DependencyPruner resets
        the path's annotation (dependency_pruner.py:320-340)."""
        if not creation:
            self.module_query("MutationPruner", [self.c.app("bvugt", self.value, self.k(0))])
        self.deps.world_state_added(creation)

    def _exec(self, max_steps: int) -> str:
        code, stack, mem = self.code, [], {}
        pc, steps = 0, 0

        def pop():
            if not stack:
                raise Halt("stack underflow")
            return stack.pop()

        def popbv():
            return self.bv(pop())

        def conc(x) -> int:
            return int(self.val(self.bv(x)))

        def mbyte(i):
            return mem.get(i) or self.k(0, 8)

        def mload(off):
            return self.app("concat", *[mbyte(off + i) for i in range(32)])

        def mstore(off, v):
            v = self.bv(v)
            for i in range(32):
                mem[off + i] = self.app("extract", v, params=(255 - 8 * i, 248 - 8 * i))

        def arith(name, kind, cond_of):
            x, y = popbv(), popbv()
            r = self.app(name, x, y)
            if cond_of is not None:
                self.annotate(kind, x, r, cond_of(x, y))
            stack.append(r)

        while True:
            steps += 1
            if steps > max_steps:
                raise Unsupported("step limit")
            if pc >= len(code):
                self.tx_end_queries()
                return "STOP"
            op = code[pc]
            if not isinstance(op, int):
                raise Unsupported(f"symbolic opcode byte at {pc}")
            self.pc = pc
            pc += 1
            a = self.app
            if op == 0x00:
                self.deps.tx_end()
                self.tx_end_queries()
                return "STOP"
            elif op == 0x01:   # integer.py:140-145 Not(BVAddNoOverflow(op0, op1, False))
                arith("bvadd", "addition", lambda x, y: a("not", a("=", a(
                    "extract", a("bvadd", a("zero_extend", x, params=(1,)), a("zero_extend", y, params=(1,))),
                    params=(256, 256)), self.k(0, 1))))
            elif op == 0x02:   # :147-151 Not(BVMulNoOverflow(op0, op1, False))
                arith("bvmul", "multiplication", lambda x, y: a("not", a("bvumul_noovfl", x, y)))
            elif op == 0x03:   # :153-157 Not(BVSubNoUnderflow(op0, op1, False)) = Not(op1 <=u op0)
                arith("bvsub", "subtraction", lambda x, y: a("not", a("bvule", y, x)))
            elif op in (0x04, 0x05, 0x06, 0x07):   # DIV SDIV MOD SMOD: concrete-zero divisor -> 0
                x, y = popbv(), popbv()
                name = {0x04: "bvudiv", 0x05: "bvsdiv", 0x06: "bvurem", 0x07: "bvsrem"}[op]
                stack.append(self.k(0) if (y.op == "const" and y.val == 0) else a(name, x, y))
            elif op == 0x0A:   # EXP: the Power UF (exponent_function_manager.py)
                b, e = popbv(), popbv()
                stack.append(self.power(b, e))
            elif op == 0x10:
                stack.append(a("bvult", popbv(), popbv()))
            elif op == 0x11:
                stack.append(a("bvugt", popbv(), popbv()))
            elif op == 0x12:
                stack.append(a("bvslt", popbv(), popbv()))
            elif op == 0x13:
                stack.append(a("bvsgt", popbv(), popbv()))
            elif op == 0x14:
                stack.append(a("=", self.bv(pop()), self.bv(pop())))
            elif op == 0x15:
                x = pop()
                e = a("not", x) if x.width == BOOL else a("=", x, self.k(0))
                stack.append(a("ite", e, self.k(1), self.k(0)) if e.op != "const" else self.k(e.val))
            elif op == 0x16:
                stack.append(a("bvand", popbv(), popbv()))
            elif op == 0x17:
                stack.append(a("bvor", popbv(), popbv()))
            elif op == 0x18:
                stack.append(a("bvxor", popbv(), popbv()))
            elif op == 0x19:
                stack.append(a("bvnot", popbv()))
            elif op == 0x1A:   # BYTE (concrete index)
                i, v = conc(pop()), popbv()
                stack.append(self.k(0) if i >= 32 else
                             a("concat", self.k(0, 248), a("extract", v, params=(255 - 8 * i, 248 - 8 * i))))
            elif op in (0x1B, 0x1C, 0x1D):
                sh, v = popbv(), popbv()
                stack.append(a({0x1B: "bvshl", 0x1C: "bvlshr", 0x1D: "bvashr"}[op], v, sh))
            elif op == 0x20:
                off, ln = conc(pop()), conc(pop())
                data = a("concat", *[mbyte(off + i) for i in range(ln)]) if ln else self.k(0, 8)
                stack.append(self.sha3(data) if ln else self.k(0xC5D2460186F7233C927E7DB2DCC703C0E500B653CA82273B7BFAD8045D85A470))
            elif op == 0x30:
                stack.append(self.k(CONTRACT))
            elif op == 0x31:   # BALANCE (instructions.py:903-920)
                addr = popbv()
                if addr.op == "const":
                    if addr.val not in self.accounts:
                        raise Unsupported("BALANCE of an account outside the world state")
                    stack.append(a("select", self.balance, addr))
                else:
                    bal = self.k(0)
                    for acct in self.accounts:
                        bal = a("ite", a("=", addr, self.k(acct)), a("select", self.balance, self.k(acct)), bal)
                    stack.append(bal)
            elif op in (0x32, 0x33):   # ORIGIN, CALLER: the transaction's sender (transaction/symbolic.py:121-131)
                stack.append(self.sender)
            elif op == 0x34:
                stack.append(self.value)
            elif op == 0x35:
                off = popbv()
                stack.append(a("concat", *[self._calldata_byte(a("bvadd", off, self.k(i)) if i else off)
                                           for i in range(32)]))
            elif op == 0x36:
                stack.append(self.cdsize)
            elif op == 0x37:   # CALLDATACOPY (concrete destination and size)
                if self.inp.creation:   # a no-op in a creation (instructions.py:885-887)
                    pop(), pop(), pop()
                    continue
                dst, src, ln = conc(pop()), popbv(), conc(pop())
                for i in range(ln):
                    mem[dst + i] = self._calldata_byte(a("bvadd", src, self.k(i)) if i else src)
            elif op == 0x38:
                if self.inp.creation:
                    # instructions.py:980-993: the code plus 0x200 bytes of symbolic
                    # constructor arguments, calldatasize pinned to that
                    n = len(code) + 0x200
                    self.constraints.append(a("=", self.cdsize, self.k(n)))
                    # the concrete choice follows the pin (the argument bytes lead the calldata)
                    self.model[f"{self.tx}_calldatasize"] = n
                    self.vals.clear()
                    stack.append(self.k(n))
                else:
                    stack.append(self.k(len(code)))
            elif op == 0x39:   # CODECOPY (instructions.py:1065-1130; concrete operands)
                dst, src, ln = conc(pop()), conc(pop()), conc(pop())
                if self.inp.creation and src >= len(code):
                    # creation code past its end is the symbolic calldata (:1078-1092)
                    off = self.k(src - len(code))
                    for i in range(ln):
                        mem[dst + i] = self._calldata_byte(a("bvadd", off, self.k(i)) if i else off)
                else:
                    for i in range(ln):
                        b = code[src + i] if src + i < len(code) else 0
                        mem[dst + i] = self.k(b, 8) if isinstance(b, int) else b
            elif op == 0x3A:
                stack.append(self.c.var(f"gas_price{self.tx}", 256))
            elif op == 0x3D:   # RETURNDATASIZE, no call returned data (instructions.py:1350-1365)
                stack.append(self._env_leaf("returndatasize", 0) if self.returndata is None
                             else self.k(len(self.returndata)))
            elif op == 0x3E:   # RETURNDATACOPY with no return data: a no-op (:1336-1337)
                dst, src, ln = pop(), pop(), pop()
                if self.returndata is not None:
                    raise Unsupported("RETURNDATACOPY of real return data")
            elif op == 0x40:   # BLOCKHASH (instructions.py:1369-1380) + PredictableVars' hooks
                stack.append(self._blockhash(pop()))
            elif op == 0x41:
                stack.append(self._predictable("coinbase", self._env_leaf("coinbase", 0)))
            elif op == 0x42:   # TIMESTAMP (instructions.py:1393-1400)
                stack.append(self._predictable("timestamp", self._env_leaf("timestamp", 1_600_000_000)))
            elif op == 0x43:   # NUMBER: environment.block_number (environment.py:47)
                stack.append(self._predictable("number", self.leaf("block_number", 10_000_000)))
            elif op == 0x44:
                stack.append(self._env_leaf("block_difficulty", 0))
            elif op == 0x45:   # GASLIMIT: the transaction's concrete gas limit
                stack.append(self.k(8_000_000))
            elif op == 0x46:
                stack.append(self.leaf("chain_id", 1))
            elif op == 0x47:   # SELFBALANCE (instructions.py:959-967)
                stack.append(a("select", self.balance, self.k(CONTRACT)))
            elif op == 0x50:
                pop()
            elif op == 0x51:
                stack.append(mload(conc(pop())))
            elif op == 0x52:
                off, v = conc(pop()), pop()
                mstore(off, v)
            elif op == 0x53:
                off, v = conc(pop()), popbv()
                mem[off] = a("extract", v, params=(7, 0))
            elif op == 0x54:
                key = popbv()
                self.deps.sload(key)          # DependencyPruner SLOAD pre hook
                stack.append(a("select", self.storage, key))
            elif op == 0x55:
                key, v = popbv(), popbv()
                self.deps.sstore(key)         # DependencyPruner SSTORE pre hook
                self.mutated = True           # MutationPruner SSTORE pre hook (mutation_pruner.py:45-47)
                self.collect(v)
                self.storage = a("store", self.storage, key, v)
            elif op == 0x56:
                dest = conc(pop())
                if dest not in self.jumpdests:
                    raise Halt("bad jump")
                pc = dest
                if not self.deps.block(self, dest):   # DependencyPruner JUMP post hook
                    return "PRUNED"
            elif op == 0x57:
                dest, cond = conc(pop()), pop()
                if self.pred.get(cond.id):
                    # PredictableVars JUMPI pre hook (dependence_on_predictable_vars.py:68-82):
                    # get_transaction_sequence(state, world constraints)
                    self.module_query("PredictableVars/jumpi", [])
                self.collect(cond)
                if cond.width == BOOL:
                    pos, neg = cond, a("not", cond)
                else:
                    pos, neg = a("not", a("=", cond, self.k(0))), a("=", cond, self.k(0))
                taken = bool(self.val(pos))
                if pos.op != "const":
                    base = self.constraints
                    for succ, follow in ((neg, not taken), (pos, taken)):
                        if succ is pos and dest not in self.jumpdests:
                            continue
                        self.constraints = base + [succ]
                        qset = self.query_set()
                        kc = qset[-1] if len(qset) > len([x for x in self.constraints
                                                          if not (x.op == "const" and x.val)]) else None
                        self.run_log.queries.append(Query(self.tx, pc - 1, follow, qset,
                                                          True if follow else None, kc))
                    self.constraints = base + [pos if taken else neg]
                if taken:
                    if dest not in self.jumpdests:
                        raise Halt("bad jump")
                    pc = dest
                if not self.deps.block(self, pc):    # DependencyPruner JUMPI post hook (the followed successor)
                    return "PRUNED"
            elif op == 0x58:
                stack.append(self.k(pc - 1))
            elif op == 0x59:
                stack.append(self.k((max(mem) + 32) // 32 * 32 if mem else 0))
            elif op == 0x5A:   # GAS: a fresh symbol (instructions.py:1697-1705)
                stack.append(self._env_leaf("gas", 2_000_000))
            elif op == 0x5B:
                pass
            elif op == 0x5F:
                stack.append(self.k(0))
            elif 0x60 <= op <= 0x7F:
                n = op - 0x5F
                bs = [code[pc + i] if pc + i < len(code) else 0 for i in range(n)]
                if all(isinstance(b, int) for b in bs):
                    stack.append(self.k(int.from_bytes(bytes(bs), "big")))
                else:   # a patched immutable (instructions.py:277-310 push_ of a symbolic argument)
                    v = a("concat", *[self.k(b, 8) if isinstance(b, int) else b for b in bs])
                    stack.append(v if v.width == 256 else a("concat", self.k(0, 256 - v.width), v))
                pc += n
            elif 0x80 <= op <= 0x8F:
                d = op - 0x7F
                if len(stack) < d:
                    raise Halt("stack underflow")
                stack.append(stack[-d])
            elif 0x90 <= op <= 0x9F:
                d = op - 0x8F
                if len(stack) < d + 1:
                    raise Halt("stack underflow")
                stack[-d - 1], stack[-1] = stack[-1], stack[-d - 1]
            elif 0xA0 <= op <= 0xA4:   # LOGn
                pop(), pop()
                for _ in range(op - 0xA0):
                    pop()
            elif op in (0xF1, 0xF2, 0xF4, 0xFA):
                self._call(op, stack, pop, popbv)
            elif op == 0xF3:
                off, ln = conc(pop()), conc(pop())
                data = [mbyte(off + i) for i in range(ln)]
                for x in data:
                    self.collect(x)
                self.deps.tx_end()
                self.tx_end_queries()
                if all(x.op == "const" for x in data):
                    self.returned = bytes(x.val for x in data)
                else:   # symbolic bytes: immutables patched into the runtime code
                    self.returned = [x.val if x.op == "const" else x for x in data]
                return "RETURN"
            elif op == 0xFD:
                off, ln = pop(), pop()
                if self._assertion_failure(off, ln, mbyte):
                    # Exceptions REVERT pre hook (exceptions.py:58-84): a Panic(0x01) revert
                    self.module_query("Exceptions", [])
                return "REVERT"
            elif op == 0xFE:
                self.module_query("Exceptions", [])   # Exceptions INVALID pre hook (exceptions.py:62-84)
                return "INVALID"
            elif op == 0xFF:
                self._selfdestruct(popbv())
                return "SELFDESTRUCT"
            else:
                raise Unsupported(f"opcode 0x{op:02x} at {pc - 1}")

    def _call(self, op: int, stack, pop, popbv) -> None:
        """CALL (0xF1), CALLCODE (0xF2), DELEGATECALL (0xF4), STATICCALL (0xFA)
        to a symbolic callee: an account with no code, so an ether transfer and
        a fresh return value (instructions.py:1960-2000, 2194-2237, 2335-2379;
        call.py:140-143).  The detection modules' hooks run around it."""
        if len(stack) < (7 if op in (0xF1, 0xF2) else 6):
            raise Halt("stack underflow")
        a = self.app
        gas, to = self.bv(stack[-1]), self.bv(stack[-2])
        if op in (0xF1, 0xFA):
            self.deps.call()           # DependencyPruner CALL / STATICCALL pre hooks (dependency_pruner.py:258-270)
            self.mutated = True        # MutationPruner CALL / STATICCALL pre hooks (mutation_pruner.py:52-58)
        if op == 0xF1:
            # ExternalCalls (CALL pre hook): _analyze_state's constraint set,
            # Constraints([UGT(gas, 2300), to == ATTACKER]) + world constraints,
            # handed to get_transaction_sequence (external_calls.py:75-82); and
            # the shape of _is_precompile_call (:29-43), world constraints +
            # Or(to <s 1, to >s PRECOMPILE_COUNT = 9) (natives.py:253-265)
            # (defined in v0.23.0 but not called by the module)
            if to.op != "const":
                self.module_query("ExternalCalls/user_supplied",
                                  [a("bvugt", gas, self.k(2300)), a("=", to, self.k(ACTORS["ATTACKER"]))], first=True)
                self.module_query("ExternalCalls/precompile",
                                  [a("or", a("bvslt", to, self.k(1)), a("bvsgt", to, self.k(9)))])
        if op in (0xF1, 0xF4, 0xF2):
            # StateChangeAfterCall pre hook (state_change_external_calls.py:183-197, 119-140)
            v3 = self.bv(stack[-3])
            if v3.op != "const":
                self.module_query("StateChangeAfterCall/balance_change", [a("bvsgt", v3, self.k(0))])
            self.module_query("StateChangeAfterCall/external_call", [
                a("bvugt", gas, self.k(2300)), a("or", a("bvsgt", to, self.k(16)), a("=", to, self.k(0)))])
            self.module_query("StateChangeAfterCall/attacker_callee", [a("=", to, self.k(ACTORS["ATTACKER"]))])
        if op == 0xF1:
            self.collect(self.bv(stack[-3]))      # integer.py:_handle_call
        pop(), pop()
        value = popbv() if op in (0xF1, 0xF2) else self.k(0)
        for _ in range(4):
            pop()
        if to.op == "const":
            raise Unsupported("call to a concrete address")
        self._transfer(self.k(CONTRACT), to, value)
        stack.append(self._env_leaf(f"retval_{self.pc}", self.inp.retvals.get(self.pc, self.inp.retvals.get(-1, 1))))
        if op in (0xF1, 0xFA):
            # EtherThief post hook (ether_thief.py:60-76)
            att = self.k(ACTORS["ATTACKER"])
            self.module_query("EtherThief", [
                a("bvugt", a("select", self.balance, att), a("select", self.balance0, att)),
                a("=", self.sender, att), self.c.true()])


class DependencyPruner:
    """``laser/plugin/plugins/dependency_pruner.py`` restated on the one path a
    concolic run follows (a default-loaded plugin; A10 feasibility caller).

    Plugin state (``:92-103``): ``iteration`` (+1 at every symbolic message
    call, ``start_sym_trans :204-206``; 0 after a creation's world state,
    ``:325-328``), ``sloads_on_path`` / ``sstores_on_path`` / ``calls_on_path``
    keyed by block address.  The path's ``DependencyAnnotation``
    (``plugin_annotations.py:26-72``): ``storage_loaded``, ``storage_written``
    (per iteration), ``has_call``, ``path``, ``blocks_seen``; it is carried to
    the next transaction through the world state (``:22-50``) with ``path``
    and ``storage_loaded`` reset (``:330-340``).

    At every JUMP / JUMPI post hook (``:208-228``) from iteration 2 on, a
    block already seen asks ``wanna_execute`` (``:146-200``): for each storage
    location written in the previous transaction, ``get_model((location ==
    dependency,))`` over the locations read on paths through the block, then
    over this path's loads; the first SAT keeps the state, none prunes it
    (``PluginSkipState``).  The queries are TUPLES: no keccak conditions
    (``model.py:35-36``), so keccak UF terms reach the engine unconstrained.

    Not restated: the branch at ``:170-177`` (``address in
    self.storage_accessed_global``), a membership test of an int block
    address in a set of z3 BitVec keys, which holds only on a hash collision
    (and then compares two ints as a Python bool)."""

    def __init__(self):
        self.iteration = 0
        self.sloads_on_path: Dict[int, List[Node]] = {}
        self.sstore_blocks: set = set()          # sstores_on_path's keys (update_calls reads only those)
        self.calls_on_path: set = set()
        self.asked: Dict[int, Optional[bool]] = {}   # eq node id -> answer (get_model's lru_cache)
        self.reset_annotation()

    def reset_annotation(self):
        self.storage_loaded: List[Node] = []
        self.storage_written: Dict[int, List[Node]] = {}
        self.has_call = False
        self.path: List[int] = [0]
        self.blocks_seen: set = set()

    def snapshot(self):
        return (list(self.storage_loaded), {k: list(v) for k, v in self.storage_written.items()}, self.has_call,
                list(self.path), set(self.blocks_seen))

    def restore(self, snap):
        (self.storage_loaded, self.storage_written, self.has_call, self.path, self.blocks_seen) = snap

    def _sloads(self, loc: Node) -> None:
        for a in self.path:
            lst = self.sloads_on_path.setdefault(a, [])
            if not any(x is loc for x in lst):
                lst.append(loc)

    def sload(self, loc: Node) -> None:         # :244-256
        if not any(x is loc for x in self.storage_loaded):
            self.storage_loaded.append(loc)
        self._sloads(loc)

    def sstore(self, loc: Node) -> None:        # :236-242
        self.sstore_blocks.update(self.path)
        lst = self.storage_written.setdefault(self.iteration, [])
        if not any(x is loc for x in lst):
            lst.append(loc)

    def _calls(self) -> None:                   # update_calls :131-140
        self.calls_on_path.update(a for a in self.path if a in self.sstore_blocks)

    def call(self) -> None:                     # :258-270
        self._calls()
        self.has_call = True

    def tx_end(self) -> None:                   # STOP / RETURN pre hooks, _transaction_end :280-297
        for loc in self.storage_loaded:
            self._sloads(loc)
        # `for index in annotation.storage_written`: the dict's keys (iterations)
        self.sstore_blocks.update(self.path)
        if self.has_call:
            self._calls()

    def world_state_added(self, creation: bool) -> None:   # :320-340
        if creation:
            self.iteration = 0
            return
        self.path = [0]
        self.storage_loaded = []

    def block(self, m: "ConcolicLaser", address: int) -> bool:
        """JUMP / JUMPI post hook on the followed successor: False = pruned."""
        self.path.append(address)
        if self.iteration < 2:
            return True
        if address not in self.blocks_seen:
            self.blocks_seen.add(address)
            return True
        if address in self.calls_on_path:
            return True
        if address not in self.sloads_on_path:
            return False
        deps = self.sloads_on_path[address]
        for loc in self.storage_written.get(self.iteration - 1, []):
            for dep in list(deps) + list(self.storage_loaded):
                if self._ask(m, loc, dep):
                    return True
        return False

    def _ask(self, m: "ConcolicLaser", loc: Node, dep: Node) -> bool:
        """get_model((location == dependency,)): identical or constant pairs
        are decided here (z3 answers them at once, nothing for the engine);
        a recorded pair keeps the state unless it is `t + j == t + k` (j != k).
        z3's answer on the others is unknown here (SAT whenever a keccak UF is
        involved: the tuple carries no keccak conditions)."""
        if loc is dep:
            return True
        eq = m.c.app("=", loc, dep)
        if eq.id in self.asked:
            return self.asked[eq.id] is not False
        ans = m.tuple_query("DependencyPruner", [eq]) if not (loc.op == "const" and dep.op == "const") \
            else loc.val == dep.val
        if ans is None:
            (b1, k1), (b2, k2) = _base_offset(loc), _base_offset(dep)
            ans = False if (b1 is b2 and k1 != k2) else None
        self.asked[eq.id] = ans
        return ans is not False


def _z3_str(n: Node) -> str:
    """str() of a BitVec as z3 prints the few shapes a BLOCKHASH argument takes
    (a numeral, a symbol, symbol +/- numeral); anything else gets a stable tag."""
    if n.op == "const":
        return str(n.val)
    if n.op == "var":
        return n.name
    if n.op in ("bvadd", "bvsub") and len(n.args) == 2 and all(x.op in ("var", "const") for x in n.args):
        return f"{_z3_str(n.args[0])} {'+' if n.op == 'bvadd' else '-'} {_z3_str(n.args[1])}"
    return f"term{n.id}"


def _base_offset(n: Node) -> Tuple[Node, int]:
    """t + k (k a constant) -> (t, k); anything else -> (n, 0)."""
    if n.op == "bvadd" and len(n.args) == 2:
        a, b = n.args
        if b.op == "const":
            return a, b.val
        if a.op == "const":
            return b, a.val
    return n, 0


def _postorder(root: Node, done: Dict[int, object]) -> List[Node]:
    out, seen = [], set()
    stack = [(root, False)]
    while stack:
        n, exp = stack.pop()
        if n.id in done or n.id in seen:
            continue
        if exp:
            seen.add(n.id)
            out.append(n)
            continue
        stack.append((n, True))
        for x in n.args:
            if x.id not in done and x.id not in seen:
                stack.append((x, False))
    return out


def _merge_slices(c: Ctx, parts: List[Node]) -> List[Node]:
    """Adjacent extract slices of one term (MSB first) merge into one slice (a
    full-width slice is the term itself: a memory word read back whole), and
    adjacent numerals into one numeral, as z3's simplify does."""
    out: List[Node] = []
    for p in parts:
        if out and p.op == "extract" and out[-1].op == "extract" and p.args[0] is out[-1].args[0] \
                and out[-1].params[1] == p.params[0] + 1:
            base = p.args[0]
            hi, lo = out[-1].params[0], p.params[1]
            out[-1] = base if (hi == base.width - 1 and lo == 0) else c.app("extract", base, params=(hi, lo))
        elif out and p.op == "const" and out[-1].op == "const" and p.width != BOOL:
            out[-1] = c.const((out[-1].val << p.width) | p.val, out[-1].width + p.width)
        else:
            out.append(p)
    return out





def asm(items):
    """A tiny assembler for the SYNTHETIC contracts (tests/test_concolic_env.py,
    tools/make_laser_corpus.py): ints are opcodes, ("push", n, v) pushes, ("label", x)
    marks a JUMPDEST, ("ref", x) pushes the label's offset (PUSH1)."""
    out, fix, labels = bytearray(), [], {}
    for it in items:
        if isinstance(it, int):
            out.append(it)
        elif it[0] == "push":
            out.append(0x5F + it[1])
            out += it[2].to_bytes(it[1], "big")
        elif it[0] == "label":
            labels[it[1]] = len(out)
            out.append(0x5B)
        else:
            out.append(0x60)
            fix.append((len(out), it[1]))
            out.append(0)
    for pos, lab in fix:
        out[pos] = labels[lab]
    return bytes(out)


def check_model(constraints: List[Node], model: Dict) -> bool:
    vals = eval_nodes(constraints, model)
    return all(vals[x.id] for x in constraints)


def abi_call(selector: int, *words: int) -> bytes:
    return selector.to_bytes(4, "big") + b"".join((w & M256).to_bytes(32, "big") for w in words)


def run_sequence(code: bytes, txs: List[TxInput], storage=None, balances=None) -> Tuple[ConcolicLaser, Run]:
    m = ConcolicLaser(code, storage, balances)
    for t, inp in enumerate(txs, start=1):
        if m.deleted and not inp.creation:
            # execute_message_call skips a self-destructed contract (transaction/symbolic.py:112-114)
            m.run_log.halts.append("skipped: contract deleted")
            continue
        # a reverted (or pruned) transaction leaves no open state (svm.py
        # _execute_transactions): the next one starts from the world state
        # before it, with that state's dependency annotation
        snap = (list(m.constraints), m.storage, m.balance, m.code, m.jumpdests, m.deps.snapshot())
        try:
            res = m.contract_creation(t, inp) if inp.creation else m.message_call(t, inp)
        except Halt as e:
            res = f"halt: {e}"
        if res not in ("STOP", "RETURN", "SELFDESTRUCT"):
            m.constraints, m.storage, m.balance, m.code, m.jumpdests, dsnap = snap
            m.deps.restore(dsnap)
        else:
            m.sequence.append(t)
        m.run_log.halts.append(res)
    m.run_log.model = m.model
    return m, m.run_log
