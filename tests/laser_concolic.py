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
  conditions appended by ``get_all_constraints`` (tests/mythril_shapes.py).

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


@dataclass
class Query:
    """A feasibility query LASER would send to get_model at a JUMPI successor."""
    tx: int
    pc: int
    taken: bool                    # the successor the concrete path follows
    constraints: List[Node]        # world-state constraints + keccak conditions
    sat: Optional[bool]            # True for the followed successor; None = unknown
    keccak_cond: Optional[Node] = None   # the manager's conditions: the last element of constraints


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
        self.model: Dict = {stor_name: ArrayVal(dict(storage or {}), 0),
                            "balance": ArrayVal(dict(balances or {}), 0)}
        self.vals: Dict[int, object] = {}
        self.run_log = Run()

    # ---------------------------------------------------------------- terms
    @staticmethod
    def _jumpdests(code: bytes):
        out, i = set(), 0
        while i < len(code):
            op = code[i]
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
        """Build a term, folding what z3's simplify folds: constant operands, and
        the concat of a term's own byte slices (memory word round trips)."""
        c = self.c
        if op == "concat":
            args = _merge_slices(c, list(args))
            if len(args) == 1:
                return args[0]
        if args and all(a.op == "const" for a in args) and op not in ("select", "store"):
            t = c.app(op, *args, params=params)
            v = _eval1(t, [a.val for a in args], {})
            return c.const(v, t.width)
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
        self.model[name] = value
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
            return self.km.create_keccak(data)
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

    def query_set(self) -> List[Node]:
        """Constraints.get_all_constraints(): the world constraints + keccak conditions."""
        cond = self.km.create_conditions()
        extra = [] if (cond.op == "const" and cond.val) else [cond]
        return [x for x in self.constraints if not (x.op == "const" and x.val)] + extra

    # ---------------------------------------------------------------- transactions
    def message_call(self, tx: int, inp: TxInput, max_steps: int = 20000) -> str:
        c = self.c
        sender = self.leaf(f"sender_{tx}", inp.sender)
        value = self.leaf(f"call_value{tx}", inp.value)
        self.leaf(f"gas_price{tx}", inp.gas_price)
        size = self.leaf(f"{tx}_calldatasize", len(inp.calldata))
        self.model[f"{tx}_calldata"] = ArrayVal(dict(enumerate(inp.calldata)), 0)
        self.cd = c.array(f"{tx}_calldata", 256, 8)
        self.cdsize = size
        self.sender, self.value, self.tx = sender, value, tx
        # transaction_models.py:139-143 then transaction/symbolic.py:210-212
        self.constraints.append(self.app("bvuge", self.app("select", self.balance, sender), value))
        me = self.k(CONTRACT)
        self.balance = self.app("store", self.balance, me, self.app("bvadd", self.app("select", self.balance, me), value))
        self.balance = self.app("store", self.balance, sender,
                                self.app("bvsub", self.app("select", self.balance, sender), value))
        self.constraints.append(c.app("or", *[c.app("=", sender, self.k(a)) for a in ACTORS.values()]))
        self.vals.clear()
        for key in ("balance",):
            pass
        return self._exec(max_steps)

    def _calldata_byte(self, i: Node) -> Node:
        return self.app("ite", self.app("bvslt", i, self.cdsize), self.app("select", self.cd, i), self.k(0, 8))

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

        while True:
            steps += 1
            if steps > max_steps:
                raise Unsupported("step limit")
            if pc >= len(code):
                return "STOP"
            op = code[pc]
            pc += 1
            a = self.app
            if op == 0x00:
                return "STOP"
            elif op == 0x01:
                stack.append(a("bvadd", popbv(), popbv()))
            elif op == 0x02:
                stack.append(a("bvmul", popbv(), popbv()))
            elif op == 0x03:
                x, y = popbv(), popbv()
                stack.append(a("bvsub", x, y))
            elif op in (0x04, 0x05, 0x06, 0x07):   # DIV SDIV MOD SMOD: concrete-zero divisor -> 0
                x, y = popbv(), popbv()
                name = {0x04: "bvudiv", 0x05: "bvsdiv", 0x06: "bvurem", 0x07: "bvsrem"}[op]
                stack.append(self.k(0) if (y.op == "const" and y.val == 0) else a(name, x, y))
            elif op == 0x0A:   # EXP: concrete only (exponent_function_manager.py:39-49)
                b, e = popbv(), popbv()
                if b.op != "const" or e.op != "const":
                    raise Unsupported("symbolic EXP")
                stack.append(self.k(pow(b.val, e.val, 1 << 256)))
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
            elif op == 0x31:
                stack.append(a("select", self.balance, popbv()))
            elif op in (0x32, 0x33):
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
                dst, src, ln = conc(pop()), popbv(), conc(pop())
                for i in range(ln):
                    mem[dst + i] = self._calldata_byte(a("bvadd", src, self.k(i)) if i else src)
            elif op == 0x38:
                stack.append(self.k(len(code)))
            elif op == 0x3A:
                stack.append(self.c.var(f"gas_price{self.tx}", 256))
            elif op in (0x42, 0x43):   # TIMESTAMP, NUMBER: fresh symbols (global_state.py:126-136)
                stack.append(self.leaf("timestamp" if op == 0x42 else "block_number", 1_600_000_000))
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
                stack.append(a("select", self.storage, popbv()))
            elif op == 0x55:
                key, v = popbv(), popbv()
                self.storage = a("store", self.storage, key, v)
            elif op == 0x56:
                dest = conc(pop())
                if dest not in self.jumpdests:
                    raise Halt("bad jump")
                pc = dest
            elif op == 0x57:
                dest, cond = conc(pop()), pop()
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
            elif op == 0x58:
                stack.append(self.k(pc - 1))
            elif op == 0x59:
                stack.append(self.k((max(mem) + 32) // 32 * 32 if mem else 0))
            elif op == 0x5A:
                stack.append(self.k(8_000_000 - steps))
            elif op == 0x5B:
                pass
            elif 0x60 <= op <= 0x7F:
                n = op - 0x5F
                stack.append(self.k(int.from_bytes(code[pc:pc + n].ljust(n, b"\0"), "big")))
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
            elif op == 0xF3:
                return "RETURN"
            elif op == 0xFD:
                return "REVERT"
            elif op == 0xFE:
                return "INVALID"
            elif op == 0xFF:
                pop()
                return "SELFDESTRUCT"
            else:
                raise Unsupported(f"opcode 0x{op:02x} at {pc - 1}")


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


def check_model(constraints: List[Node], model: Dict) -> bool:
    vals = eval_nodes(constraints, model)
    return all(vals[x.id] for x in constraints)


def abi_call(selector: int, *words: int) -> bytes:
    return selector.to_bytes(4, "big") + b"".join((w & M256).to_bytes(32, "big") for w in words)


def run_sequence(code: bytes, txs: List[TxInput], storage=None, balances=None) -> Tuple[ConcolicLaser, Run]:
    m = ConcolicLaser(code, storage, balances)
    for t, inp in enumerate(txs, start=1):
        # a reverted transaction leaves no open state (svm.py _execute_transactions):
        # the next one starts from the world state before it
        snap = (list(m.constraints), m.storage, m.balance)
        try:
            res = m.message_call(t, inp)
        except Halt as e:
            res = f"halt: {e}"
        if res not in ("STOP", "RETURN", "SELFDESTRUCT"):
            m.constraints, m.storage, m.balance = snap
        m.run_log.halts.append(res)
    m.run_log.model = m.model
    return m, m.run_log
