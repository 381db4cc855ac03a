"""Constraint DAG -> witness-engine bytecode.

Input: the conjuncts of a Mythril constraint set (``Constraints`` list,
``mythril/laser/ethereum/state/constraints.py:10-108``) as IR terms.  Output:
a :class:`Program` — straight-line bytecode for ``csrc/mw_interp.h``, a
constant pool, the leaf (free-variable) table with candidate pools, and the
algorithmic op count per candidate (SURVEY.md §8(d) cost table).

Passes
  1. flatten top-level ``and`` into conjuncts (each becomes one CHECK so a
     wavefront can stop at the first conjunct no lane satisfies);
  2. lower every term to machine ops on virtual registers (W class: widths
     33..256 in 8 limbs; N class: widths 1..32, Bools are width-1 N values);
  3. schedule conjunct by conjunct in operand-first order, leaves at first use;
  4. allocate the MW_NW W slots / MW_NN N slots with Belady (furthest next use)
     eviction, emitting SPILL/FILL to a per-lane spill area when needed;
  5. encode.

Anything outside the supported vocabulary raises :class:`Unsupported`, which
the drop-in ``get_model`` turns into "fall back to z3" (fail closed).
"""
from __future__ import annotations

import math
import os
import zlib
from array import array
from dataclasses import dataclass, field
from typing import Callable, Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np

from . import isa
from .ir import BOOL, Node, topo


# candidate-index bits available to exhaustive pool digits; the bits above
# them enumerate "rounds" that re-draw every RANDOM entry
INDEX_FIELD_BITS = 40


class Unsupported(Exception):
    """The formula uses something the GPU path does not evaluate (-> z3)."""


# --------------------------------------------------------------------------- machine IR
class VReg:
    __slots__ = ("id", "cls")

    def __init__(self, vid: int, cls: str):
        self.id = vid
        self.cls = cls

    def __repr__(self):  # pragma: no cover
        return f"%{self.cls}{self.id}"


class Const:
    __slots__ = ("value", "cls")

    def __init__(self, value: int, cls: str):
        self.value = value
        self.cls = cls

    def __repr__(self):  # pragma: no cover
        return f"${self.value:#x}"


@dataclass
class MInsn:
    op: str
    width: int = 0
    dst: Optional[VReg] = None
    srcs: List[object] = field(default_factory=list)
    imm: int = 0
    remat: bool = False   # recomputation of a term from an earlier conjunct (jit.py fences its inputs)
    chain: bool = False   # W_CDINS whose result's only use is the next W_CDINS's acc (MW_FLAG_CHAIN)


def cls_of(width: int) -> str:
    return "N" if width <= isa.NARROW_MAX else "W"


def _w(n: Node) -> int:
    """Machine width of a term (Bool -> 1)."""
    return 1 if n.width == BOOL else n.width


# --------------------------------------------------------------------------- leaves / pools
@dataclass
class LeafSpec:
    """Candidate generator for one free variable (DESIGN.md "Candidate space")."""
    name: str
    width: int
    pool: Optional[List[Optional[int]]] = None   # None entry = RANDOM; len must be 2**k
    shift: int = 0
    bits: int = 0
    hashed: bool = False         # pool digit from a hash of the index instead of a bit-field
    stride: int = 0              # >0: bit-interleaved digit (index bits shift, shift+stride, ...)
    salt: Optional[int] = None   # Philox key salt; default crc32(name) so a variable
                                 # draws the same value in every program for an index
    tie: Optional[str] = None    # copy this leaf's digit layout (bytes of one ABI word
                                 # pick the same pool entry: pools.harvest word groups)

    def key_salt(self) -> int:
        return self.salt if self.salt is not None else zlib.crc32(self.name.encode()) & 0xFFFFFFFF


@dataclass
class Program:
    code: np.ndarray
    consts: np.ndarray
    leaves: np.ndarray
    pool: np.ndarray
    n_spill: int
    n_trace_rows: int
    n_input_rows: int
    ops_per_eval: int
    leaf_specs: List[LeafSpec]
    leaf_nodes: List[Node]
    trace_map: Dict[int, Tuple[int, str]]
    n_insn: int
    n_conjuncts: int
    stats: Dict[str, int] = field(default_factory=dict)
    ssa: List[MInsn] = field(default_factory=list)   # machine IR before slot allocation (jit.py)
    # natively compiled programs (ccompile.py) carry no machine IR; this builds it on first use
    ssa_build: Optional[Callable[[], List[MInsn]]] = None
    # natively compiled programs: the record stream they were compiled from
    # (ccompile.compile_trace_native compiles the witness program from it)
    native_dag: Optional[tuple] = None

    def machine_ir(self) -> List[MInsn]:
        """The SSA machine IR the specialised kernels are generated from (jit.py)."""
        if not self.ssa and self.ssa_build is not None:
            self.ssa = self.ssa_build()
        return self.ssa

    def executed_ops(self, evals: int, st: Optional[dict] = None) -> float:
        """Algorithmic u32 ops a search of `evals` candidates executed: ops_per_eval
        with every wide division's nominal price (SURVEY §8(d) via node_cost)
        replaced by the price of the path the kernel took, from the per-wave
        counts it reports (mg_stats.lane_div_*, each x the wave's lanes):
        DIV_PRICE_* below.  st=None gives the division-free floor (no credit
        for any division)."""
        floor = evals * (self.ops_per_eval - self.stats.get("div_nominal_ops", 0))
        if not st:
            return float(floor)
        return float(floor + st.get("lane_div_full", 0) * DIV_PRICE_FULL
                     + st.get("lane_div_short", 0) * DIV_PRICE_SHORT
                     + st.get("lane_div_general", 0) * DIV_PRICE_GENERAL
                     + st.get("lane_div_steps", 0) * DIV_PRICE_STEP)

    def input_rows_for(self, leaf_index: int) -> Tuple[int, int]:
        off = int(self.leaves[leaf_index * isa.LEAF_WORDS + isa.LEAF_INROW])
        return off, (self.leaf_specs[leaf_index].width + 31) // 32


# --------------------------------------------------------------------------- cost model
# Executed price of the three udivrem8 paths (csrc/mw_alu.h), in the units of
# node_cost: a 32x32->64 product is 2 ops (lo, hi), add/sub with carry 2,
# compare/select 1; the f64 digit estimates are not u32 work and are not
# counted.  Every wide division runs on 8 limbs (L = 8).
#   one digit step (multiply-subtract over 8 limbs + top-limb test): 6L + 2
#   full-width divisor: one step                                      = 50
#   one-limb divisor: 8 two-by-one steps of 14 ops, normalise/unshift = 115
#   schoolbook entry: divisor limb count (7), limb shifts of v and u
#     (3 stages x (8 + 16) selects), remainder unshift (3 x 8), zero-digit
#     tests (8 x 2)                                                    = 119
#   schoolbook digit step: as the full-width step                      = 50
DIV_PRICE_STEP = 6 * 8 + 2
DIV_PRICE_FULL = DIV_PRICE_STEP
DIV_PRICE_SHORT = 8 * 14 + 3
DIV_PRICE_GENERAL = 7 + 3 * (8 + 16) + 3 * 8 + 8 * 2


def node_cost(n: Node) -> int:
    """Algorithmic u32 ops to evaluate one node once."""
    op = n.op
    if op in ("const", "var", "array", "apply"):
        return 0
    k = len(n.args)
    if n.width == BOOL and op in ("and", "or", "not", "xor", "=>"):
        return max(k, 1)
    if op == "ite":
        return max(1, (_w(n) + 31) // 32)
    if op in ("=", "distinct") and n.args and n.args[0].width == BOOL:
        return k
    aw = _w(n.args[0]) if n.args else _w(n)
    L = (aw + 31) // 32
    Lo = (_w(n) + 31) // 32
    if op in ("bvadd", "bvsub", "bvand", "bvor", "bvxor"):
        return L * max(k - 1, 1)
    if op == "bvaddc":
        return L
    if op in ("bvneg", "bvnot"):
        return L
    if op in ("bvnand", "bvnor", "bvxnor"):
        return 2 * L
    if op in ("=", "distinct"):
        return 2 * L * max(k - 1, 1)
    if op in ("bvult", "bvule", "bvugt", "bvuge", "bvslt", "bvsle", "bvsgt", "bvsge"):
        return L + 1
    if op in ("extract", "concat", "zero_extend", "sign_extend", "repeat", "rotate_left",
              "rotate_right"):
        return Lo
    if op in ("bvshl", "bvlshr", "bvashr"):
        return 2 * L + L * max(1, math.ceil(math.log2(L))) if L > 1 else 2
    if op == "bvmul":
        return 2 * L * (L + 1) * max(k - 1, 1)
    if op == "bvumul_noovfl":
        return 4 * L * L + L
    if op in ("bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod"):
        if L == 1:
            base = 20
        else:
            lg = max(1, math.ceil(math.log2(L)))
            base = L * (6 * L + 20) + 3 * (2 * L + L * lg)
        return base + (4 * L if op in ("bvsdiv", "bvsrem", "bvsmod") else 0)
    if op == "bvcomp":
        return 2 * L
    return L


# --------------------------------------------------------------------------- compiler
class _Lowerer:
    def __init__(self):
        self.insns: List[MInsn] = []
        self.memo: Dict[int, object] = {}
        self.memo_scope: Dict[int, int] = {}   # node id -> conjunct in which it was computed
        self.memo_at: Dict[int, int] = {}      # node id -> instruction count when it was computed
        self.scope = 0
        self.nv = 0
        self.leaf_index: Dict[str, int] = {}
        self.leaf_nodes: List[Node] = []
        self.trace_req: Dict[int, Node] = {}
        self.trace_emitted: Dict[int, object] = {}

    def vreg(self, cls: str) -> VReg:
        self.nv += 1
        return VReg(self.nv, cls)

    def emit(self, op: str, width: int, srcs: Sequence[object] = (), imm: int = 0) -> VReg:
        dcls = isa.SHAPES[op][0]
        d = self.vreg(dcls) if dcls else None
        self.insns.append(MInsn(op, width, d, list(srcs), imm))
        return d

    def emit_void(self, op: str, width: int, srcs: Sequence[object] = (), imm: int = 0):
        self.insns.append(MInsn(op, width, None, list(srcs), imm))

    @staticmethod
    def k(value: int, width: int) -> Const:
        return Const(value & ((1 << width) - 1), cls_of(width))

    # ---- helpers producing values of a given machine width
    def as_cls(self, v, width: int, want: str):
        """Make sure operand v (a value of `width`) sits in class `want`."""
        have = v.cls
        if have == want:
            return v
        if want == "W":  # N -> W zero extension
            if isinstance(v, Const):
                return Const(v.value, "W")
            return self.emit("W_ZEXTN", max(width, 33), [v])
        raise Unsupported("narrowing class change")

    # Cheap terms over leaves/constants (e.g. ``bvor(x, 1)``, ``extract(x)``) are
    # hash-consed across the whole DAG; keeping one computed copy live from its
    # first to its last use costs 8 registers for the whole span.  Such a term
    # is recomputed instead when its last computation is in an earlier conjunct
    # or more than REMAT_DISTANCE instructions back (REMAT_MAX_COST u32 ops at
    # most).
    REMAT_MAX_COST = 16
    REMAT_DISTANCE = 32

    def _fresh(self, m: Node) -> bool:
        if m.id not in self.memo:
            return False
        if m.op in ("var", "const") or not m.args or node_cost(m) > self.REMAT_MAX_COST:
            return True
        if not all(a.op in ("var", "const") for a in m.args):
            return True
        if (self.memo_scope.get(m.id, self.scope) == self.scope
                and len(self.insns) - self.memo_at.get(m.id, 0) <= self.REMAT_DISTANCE):
            return True
        del self.memo[m.id]  # recompute here
        return False

    def lower(self, n: Node):
        if self._fresh(n):
            return self.memo[n.id]
        # operand-first (post-order) without recursion: DAGs can be thousands deep
        stack = [(n, False)]
        while stack:
            m, expanded = stack.pop()
            if expanded:
                if m.id not in self.memo:
                    self._lower_one(m)
                continue
            if self._fresh(m):
                continue
            stack.append((m, True))
            if self._lazy_concat(m):
                continue   # parts are lowered one by one as they are inserted (_concat_lazy)
            for a in reversed(m.args):
                if not self._fresh(a):
                    stack.append((a, False))
        return self.memo[n.id]

    @staticmethod
    def _lazy_concat(m: Node) -> bool:
        return m.op == "concat" and cls_of(_w(m)) == "W" and _w(m) <= isa.MAX_WIDTH

    def _lower_one(self, n: Node):
        if n.id in self.memo:
            return self.memo[n.id]
        first = len(self.insns)
        v = self._lower(n)
        if n.id in self.memo_scope:  # lowered before, in an earlier conjunct
            for ins in self.insns[first:]:
                ins.remat = True
        self.memo[n.id] = v
        self.memo_scope[n.id] = self.scope
        self.memo_at[n.id] = len(self.insns)
        if n.id in self.trace_req and n.id not in self.trace_emitted:
            self.trace_emitted[n.id] = v
            cls = v.cls
            self.insns.append(MInsn("STORE_W" if cls == "W" else "STORE_N", _w(n), None, [v],
                                    imm=-(n.id + 1)))  # row patched at encode time
        return v

    def _bin(self, op_w: str, op_n: str, width: int, a, b):
        if cls_of(width) == "W":
            return self.emit(op_w, width, [self.as_cls(a, width, "W"), self.as_cls(b, width, "W")])
        return self.emit(op_n, width, [a, b])

    def _lower(self, n: Node):
        op = n.op
        w = _w(n)
        if n.is_array:
            raise Unsupported("array term outside select (Ackermannisation pending)")
        if op == "const":
            return self.k(n.val, w)
        if op == "var":
            if w > isa.MAX_WIDTH:
                raise Unsupported("free variable wider than 256 bits")
            if n.name not in self.leaf_index:
                self.leaf_index[n.name] = len(self.leaf_nodes)
                self.leaf_nodes.append(n)
            li = self.leaf_index[n.name]
            return self.emit("LEAF_W" if cls_of(w) == "W" else "LEAF_N", w, [], imm=li)
        if w > isa.MAX_WIDTH or any(_w(a) > isa.MAX_WIDTH for a in n.args if not a.is_array):
            raise Unsupported(f"{op} wider than 256 bits")
        if op in ("select", "store", "apply", "const_array"):
            raise Unsupported(f"{op} (Ackermannisation pending)")

        if self._lazy_concat(n):
            return self._concat_lazy(n)
        args = [self.lower(a) for a in n.args]
        # ---------------- Bool connectives (width-1 N values)
        if n.width == BOOL:
            if op == "and":
                return self._fold("N_AND", 1, args)
            if op == "or":
                return self._fold("N_OR", 1, args)
            if op == "xor":
                return self._fold("N_XOR", 1, args)
            if op == "not":
                return self.emit("N_XOR", 1, [args[0], self.k(1, 1)])
            if op == "=>":   # a => b  ==  a <=u b on Bools: one instruction instead of not + or
                return self.emit("N_ULEN", 1, [args[0], args[1]])
            if op in ("=", "distinct"):
                aw = _w(n.args[0])
                if n.args[0].is_array:
                    raise Unsupported("array equality")
                pairs = []
                if op == "=":
                    for b in args[1:]:
                        pairs.append(self._eq(aw, args[0], b))
                    r = self._fold("N_AND", 1, pairs)
                    return r
                for i in range(len(args)):
                    for j in range(i + 1, len(args)):
                        e = self._eq(aw, args[i], args[j])
                        pairs.append(self.emit("N_XOR", 1, [e, self.k(1, 1)]))
                return self._fold("N_AND", 1, pairs)
            if op in ("bvult", "bvule", "bvugt", "bvuge", "bvslt", "bvsle", "bvsgt", "bvsge"):
                aw = _w(n.args[0])
                a, b = args
                base = {"bvult": ("ULT", False), "bvule": ("ULE", False), "bvugt": ("ULT", True),
                        "bvuge": ("ULE", True), "bvslt": ("SLT", False), "bvsle": ("SLE", False),
                        "bvsgt": ("SLT", True), "bvsge": ("SLE", True)}[op]
                name, swap = base
                if swap:
                    a, b = b, a
                if cls_of(aw) == "W":
                    return self.emit("N_" + name, aw, [self.as_cls(a, aw, "W"), self.as_cls(b, aw, "W")])
                return self.emit("N_" + name + "N", aw, [a, b])
            if op == "bvaddc":   # carry out of a + b (lower.py wide-arithmetic legalisation)
                aw = _w(n.args[0])
                if cls_of(aw) == "W":
                    return self.emit("N_ADDC", aw, [self.as_cls(args[0], aw, "W"), self.as_cls(args[1], aw, "W")])
                return self.emit("N_ADDCN", aw, args)
            if op == "bvumul_noovfl":
                aw = _w(n.args[0])
                return self._bin("N_UMULNO", "N_UMULNON", aw, *args) if cls_of(aw) == "W" else \
                    self.emit("N_UMULNON", aw, args)
            if op == "ite":
                return self.emit("N_ITE", 1, [args[1], args[2], args[0]])
            raise Unsupported(f"bool op {op}")

        # ---------------- bitvector ops
        C = cls_of(w)
        if op == "bvadd":
            return self._fold("W_ADD" if C == "W" else "N_ADD", w, args)
        if op == "bvmul":
            return self._fold("W_MUL" if C == "W" else "N_MUL", w, args)
        if op == "bvand":
            return self._fold("W_AND" if C == "W" else "N_AND", w, args)
        if op == "bvor":
            return self._fold("W_OR" if C == "W" else "N_OR", w, args)
        if op == "bvxor":
            return self._fold("W_XOR" if C == "W" else "N_XOR", w, args)
        if op == "bvsub":
            return self._bin("W_SUB", "N_SUB", w, *args)
        if op == "bvneg":
            return self._bin("W_SUB", "N_SUB", w, self.k(0, w), args[0])
        if op == "bvnot":
            return self.emit("W_NOT" if C == "W" else "N_NOT", w, [args[0]])
        if op in ("bvnand", "bvnor", "bvxnor"):
            inner = {"bvnand": "AND", "bvnor": "OR", "bvxnor": "XOR"}[op]
            t = self._bin("W_" + inner, "N_" + inner, w, *args)
            return self.emit("W_NOT" if C == "W" else "N_NOT", w, [t])
        if op in ("bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod"):
            s = op[2:].upper()
            return self._bin("W_" + s, "N_" + s, w, *args)
        if op in ("bvshl", "bvlshr", "bvashr"):
            a, b = args
            if isinstance(b, Const) and op != "bvashr":
                if b.value >= w:
                    return self.k(0, w)
                if b.value == 0:
                    return a
                name = ("W_" if C == "W" else "N_") + ("SHLI" if op == "bvshl" else "LSHRI")
                return self.emit(name, w, [a], imm=b.value)
            s = {"bvshl": "SHL", "bvlshr": "LSHR", "bvashr": "ASHR"}[op]
            return self._bin("W_" + s, "N_" + s, w, a, b)
        if op == "ite":
            c, a, b = args
            if C == "W":
                return self.emit("W_ITE", w, [self.as_cls(a, w, "W"), self.as_cls(b, w, "W"), c])
            return self.emit("N_ITE", w, [a, b, c])
        if op == "bvcomp":
            return self._eq(_w(n.args[0]), args[0], args[1])
        if op == "extract":
            hi, lo = n.params
            a = args[0]
            aw = _w(n.args[0])
            if isinstance(a, Const):
                return self.k(a.value >> lo, w)
            if cls_of(aw) == "W":
                if C == "N":
                    return self.emit("N_EXTRACTW", w, [a], imm=lo)
                if lo == 0 and w == aw:
                    return a
                return self.emit("W_LSHRI", w, [a], imm=lo)
            if lo == 0 and w == aw:
                return a
            return self.emit("N_LSHRI", w, [a], imm=lo)
        if op == "zero_extend":
            a = args[0]
            if isinstance(a, Const):
                return Const(a.value, C)
            return self.as_cls(a, _w(n.args[0]), C)
        if op == "sign_extend":
            a = args[0]
            aw = _w(n.args[0])
            if C == "N":
                return self.emit("N_SEXT", w, [a], imm=aw)
            if a.cls == "N":
                return self.emit("W_SEXTN", w, [a], imm=aw)
            return self.emit("W_SEXT", w, [a], imm=aw)
        if op == "concat":
            return self._concat([_w(x) for x in n.args], args, w)
        if op == "repeat":
            aw = _w(n.args[0])
            return self._concat([aw] * n.params[0], [args[0]] * n.params[0], w)
        if op in ("rotate_left", "rotate_right"):
            r = n.params[0] % w
            a = args[0]
            if r == 0:
                return a
            left = r if op == "rotate_left" else w - r
            p = "W_" if C == "W" else "N_"
            hi = self.emit(p + "SHLI", w, [a], imm=left)
            lo = self.emit(p + "LSHRI", w, [a], imm=w - left)
            return self.emit(p + "OR", w, [hi, lo])
        raise Unsupported(f"op {op}")

    def _fold(self, op: str, w: int, args):
        if len(args) == 1:
            return args[0]
        acc = args[0]
        C = "W" if op.startswith("W_") else "N"
        for b in args[1:]:
            if C == "W":
                acc = self.emit(op, w, [self.as_cls(acc, w, "W"), self.as_cls(b, w, "W")])
            else:
                acc = self.emit(op, w, [acc, b])
        return acc

    def _eq(self, aw: int, a, b):
        if cls_of(aw) == "W":
            return self.emit("N_EQ", aw, [self.as_cls(a, aw, "W"), self.as_cls(b, aw, "W")])
        return self.emit("N_EQN", aw, [a, b])

    def _concat_lazy(self, n: Node):
        """A wide concat built part by part from the least significant end, each
        part lowered right before it is inserted: an ABI word of 32 guarded
        calldata bytes keeps one byte live instead of 32, and every byte is the
        adjacent ``N_SLT, LEAF_N, N_ITE, W_INSN`` run that _fuse_checks turns
        into one W_CDINS."""
        w = _w(n)
        acc = None
        off = 0
        for part in reversed(n.args):
            pw = _w(part)
            v = self.lower(part)
            if acc is None:
                acc = Const(v.value, "W") if isinstance(v, Const) else (v if v.cls == "W" else
                                                                       self.emit("W_ZEXTN", w, [v]))
            elif isinstance(v, Const):
                if v.value:
                    acc = self.emit("W_OR", w, [self.as_cls(acc, w, "W"), Const(v.value << off, "W")])
            elif v.cls == "N":
                acc = self.emit("W_INSN", w, [self.as_cls(acc, w, "W"), v], imm=off)
            else:
                sh = self.emit("W_SHLI", w, [v], imm=off)
                acc = self.emit("W_OR", w, [self.as_cls(acc, w, "W"), sh])
            off += pw
        return acc

    def _concat(self, widths: List[int], vals: List[object], w: int):
        # first argument is most significant; build from the least significant part up
        parts = list(zip(widths, vals))[::-1]
        off = 0
        if cls_of(w) == "N":
            acc = None
            for pw, v in parts:
                if acc is None:
                    acc = v
                else:
                    sh = self.emit("N_SHLI", w, [v], imm=off) if off else v
                    acc = self.emit("N_OR", w, [acc, sh])
                off += pw
            return acc
        acc = None
        for pw, v in parts:
            if acc is None:
                if isinstance(v, Const):
                    acc = Const(v.value, "W")
                elif v.cls == "W":
                    acc = v
                else:
                    acc = self.emit("W_ZEXTN", w, [v])
            elif isinstance(v, Const):
                if v.value:
                    acc = self.emit("W_OR", w, [self.as_cls(acc, w, "W"), Const(v.value << off, "W")])
            elif v.cls == "N":
                acc = self.emit("W_INSN", w, [self.as_cls(acc, w, "W"), v], imm=off)
            else:
                sh = self.emit("W_SHLI", w, [v], imm=off)
                acc = self.emit("W_OR", w, [self.as_cls(acc, w, "W"), sh])
            off += pw
        return acc


def _flatten(conjuncts: Iterable[Node]) -> List[Node]:
    out: List[Node] = []
    stack = list(conjuncts)[::-1]
    while stack:
        c = stack.pop()
        if c.width != BOOL:
            raise Unsupported("conjunct is not Bool")
        if c.op == "and":
            stack.extend(list(c.args)[::-1])
        elif c.op == "const" and c.val:
            continue
        else:
            out.append(c)
    return out


# --------------------------------------------------------------------------- scheduling
HOIST_CAP = 16


def _uses(insns: List[MInsn]) -> Dict[int, int]:
    uses: Dict[int, int] = {}
    for ins in insns:
        for s in ins.srcs:
            if isinstance(s, VReg):
                uses[s.id] = uses.get(s.id, 0) + 1
    return uses


def _is(v, ins: MInsn) -> bool:
    return isinstance(v, VReg) and ins.dst is not None and v.id == ins.dst.id


def _fuse_checks(insns: List[MInsn]) -> List[MInsn]:
    """Interpreter superinstructions (bytecode only: ``Program.ssa`` keeps the
    unfused list for jit.py).  The interpreter is dispatch-bound,
    so the frequent Mythril shapes run as one dispatch each:

    * ``t = a <=u b; CHECK t`` (a Bool implication, ``=>`` in _lower) ->
      ``CHECK_IMP a, b``;
    * ``t = (x = y); CHECK_IMP p, t`` -> ``CHECK_IMPEQ p, x, y`` (narrow) or
      ``CHECK_IMPEQW`` (wide): C3's 2 176 congruence conjuncts
      ``(i_t = i_u) => (v_t = v_u)`` (lower.py);
    * ``c = K <s size; l = LEAF_N; b = ite(c, l, 0); acc' = acc | b << off``
      -> ``W_CDINS``: one guarded calldata byte of an ABI word
      (``If(i <s size, calldata[i], 0)``, state/calldata.py:218-231), the
      bulk of C2's program.
    Temporaries must have no other use."""
    uses = _uses(insns)
    out: List[MInsn] = []
    i = 0
    while i < len(insns):
        ins = insns[i]
        nxt = insns[i + 1] if i + 1 < len(insns) else None
        if (ins.op == "N_ULEN" and ins.width == 1 and ins.dst is not None and nxt is not None
                and nxt.op == "CHECK" and len(nxt.srcs) == 1 and _is(nxt.srcs[0], ins)
                and uses.get(ins.dst.id, 0) == 1):
            out.append(MInsn("CHECK_IMP", 1, None, list(ins.srcs)))
            i += 2
            continue
        out.append(ins)
        i += 1
    insns, out, i = out, [], 0
    uses = _uses(insns)
    while i < len(insns):
        ins = insns[i]
        nxt = insns[i + 1] if i + 1 < len(insns) else None
        if (ins.op in ("N_EQN", "N_EQ") and ins.dst is not None and nxt is not None and nxt.op == "CHECK_IMP"
                and _is(nxt.srcs[1], ins) and uses.get(ins.dst.id, 0) == 1):
            op = "CHECK_IMPEQ" if ins.op == "N_EQN" else "CHECK_IMPEQW"
            out.append(MInsn(op, ins.width, None, [nxt.srcs[0], ins.srcs[0], ins.srcs[1]]))
            i += 2
            continue
        q = insns[i:i + 4]
        if (len(q) == 4 and q[0].op == "N_SLT" and q[0].width == 256 and isinstance(q[0].srcs[0], Const)
                and isinstance(q[0].srcs[1], VReg) and q[1].op == "LEAF_N"
                and q[2].op == "N_ITE" and _is(q[2].srcs[0], q[1]) and isinstance(q[2].srcs[1], Const)
                and q[2].srcs[1].value == 0 and _is(q[2].srcs[2], q[0])
                and ((q[3].op == "W_INSN" and _is(q[3].srcs[1], q[2]))
                     or (q[3].op == "W_ZEXTN" and _is(q[3].srcs[0], q[2])))
                and uses.get(q[0].dst.id, 0) == 1 and uses.get(q[2].dst.id, 0) == 1
                and q[1].imm < (1 << 16)):
            if uses.get(q[1].dst.id, 0) > 1:
                # the byte's leaf has other uses (a congruence grid's table or
                # rows): it stays, and W_CDINS draws the same leaf again
                # itself; _hoist_cdins_leaves keeps the chain unbroken
                q[1].cdleaf = True
                out.append(q[1])
            acc = q[3].srcs[0] if q[3].op == "W_INSN" else Const(0, "W")
            off = q[3].imm if q[3].op == "W_INSN" else 0
            out.append(MInsn("W_CDINS", q[3].width, q[3].dst, [acc, q[0].srcs[1], Const(q[0].srcs[0].value, "W")],
                             imm=q[1].imm | (off << 16)))
            i += 4
            continue
        out.append(ins)
        i += 1
    out = _hoist_cdins_leaves(out)
    out = _form_grids(_fuse_keyed_premises(out))
    uses = _uses(out)
    for a, b in zip(out, out[1:]):
        if (a.op == "W_CDINS" and b.op == "W_CDINS" and a.dst is not None and uses.get(a.dst.id, 0) == 1
                and _is(b.srcs[0], a)):
            a.chain = True
    return out


def _hoist_cdins_leaves(insns: List[MInsn]) -> List[MInsn]:
    """In a run of W_CDINS links and the leaves kept beside them (_fuse_checks:
    a leaf with other uses), the leaves move to the run's start, so the links
    stay adjacent and chain (a leaf has no operands: it can move earlier)."""
    out: List[MInsn] = []
    i = 0
    while i < len(insns):
        if insns[i].op == "W_CDINS" or getattr(insns[i], "cdleaf", False):
            j = i
            while j < len(insns) and (insns[j].op == "W_CDINS" or getattr(insns[j], "cdleaf", False)):
                j += 1
            seg = insns[i:j]
            out += [x for x in seg if x.op != "W_CDINS"] + [x for x in seg if x.op == "W_CDINS"]
            i = j
        else:
            out.append(insns[i])
            i += 1
    return out


def _fuse_keyed_premises(insns: List[MInsn]) -> List[MInsn]:
    """``p = (key = K); CHECK_IMPEQ p, x, y`` -> ``CHECK_IMPEQK key, x, y, imm=K``
    for K < isa.IMPEQK_LIMIT: a congruence premise over an index key
    (lower._index_key) is compared inside the check, and the premise flags,
    one per diagonal K - k of the pair grid and live across it, are dropped
    once no other instruction reads them."""
    defs = {ins.dst.id: ins for ins in insns if ins.dst is not None}
    fused = set()
    out: List[MInsn] = []
    for ins in insns:
        p = ins.srcs[0] if ins.op == "CHECK_IMPEQ" else None
        d = defs.get(p.id) if isinstance(p, VReg) else None
        if d is not None and d.op == "N_EQN" and d.width <= 32:
            key, k = d.srcs
            if isinstance(key, Const):
                key, k = k, key
            if isinstance(key, VReg) and isinstance(k, Const) and k.value < isa.IMPEQK_LIMIT:
                out.append(MInsn("CHECK_IMPEQK", ins.width, None, [key, ins.srcs[1], ins.srcs[2]], imm=k.value))
                fused.add(d.dst.id)
                continue
        out.append(ins)
    if not fused:
        return out
    uses = _uses(out)
    return [ins for ins in out if ins.dst is None or ins.dst.id not in fused or uses.get(ins.dst.id, 0)]


GRID_MIN = 64      # keyed checks of one key before they become a table (_form_grids)
GRID_MAX_N = 32    # table entries: CHECK_GRID's c field holds n - 1 in 5 bits, the table's word in 10


def _okey(o):
    return ("v", o.id) if isinstance(o, VReg) else ("k", o.value, o.cls)


def _grid_plan(insns: List[MInsn], pos: List[int]):
    """(table operands in offset order, {row operand key: (operand, E, last position)}) for
    the keyed checks at `pos` (one key), or None unless they form a complete grid
    e(r, t) = E_r - k_t with the k_t distinct in [0, n)."""
    first: Dict[tuple, object] = {}
    adj: Dict[tuple, List[tuple]] = {}
    for p in pos:
        x, y = insns[p].srcs[1], insns[p].srcs[2]
        kx, ky = _okey(x), _okey(y)
        if kx == ky:
            return None
        for k, o in ((kx, x), (ky, y)):
            if k not in first:
                first[k] = o
                adj[k] = []
        adj[kx].append(ky)
        adj[ky].append(kx)
    # 2-colour the operands (a complete bipartite graph is connected); colour 0
    # holds the first operand met
    colour: Dict[tuple, int] = {}
    order = list(first)
    colour[order[0]] = 0
    stack = [order[0]]
    while stack:
        k = stack.pop()
        for m in adj[k]:
            if m not in colour:
                colour[m] = 1 - colour[k]
                stack.append(m)
            elif colour[m] == colour[k]:
                return None
    if len(colour) != len(order):
        return None
    sides = [[k for k in order if colour[k] == c] for c in (0, 1)]
    # the larger side that fits is the table: a store per entry is cheaper than a row
    for tside in ((0, 1) if len(sides[0]) >= len(sides[1]) else (1, 0)):
        tkeys, rkeys = sides[tside], sides[1 - tside]
        n, m = len(tkeys), len(rkeys)
        if n > GRID_MAX_N or n * m != len(pos):
            continue
        tset = set(tkeys)
        e: Dict[Tuple[tuple, tuple], int] = {}
        last: Dict[tuple, int] = {}
        ok = True
        for p in pos:
            ins = insns[p]
            kx, ky = _okey(ins.srcs[1]), _okey(ins.srcs[2])
            t, r = (kx, ky) if kx in tset else (ky, kx)
            if (t, r) in e:
                ok = False
                break
            e[(t, r)] = ins.imm
            last[r] = p
        if not ok or len(e) != n * m:
            continue
        r0 = rkeys[0]
        top = max(e[(t, r0)] for t in tkeys)
        off = {t: top - e[(t, r0)] for t in tkeys}
        if sorted(off.values()) != list(range(n)):
            continue
        rows = {}
        for r in rkeys:
            E = {e[(t, r)] + off[t] for t in tkeys}
            if len(E) != 1:
                ok = False
                break
            rows[r] = (first[r], E.pop(), last[r])
        if not ok:
            continue
        table = sorted(tkeys, key=lambda t: off[t])
        return [first[t] for t in table], rows
    return None


def _form_grids(insns: List[MInsn]) -> List[MInsn]:
    """A complete grid of keyed congruence checks over one key (C3: an ABI
    word's 32 bytes S_k at a symbolic offset against 68 concrete cells v_K,
    ``(key = E_K - k) => (S_k = v_K)``) becomes a table and one lookup per
    row: the S_k are stored to n consecutive spill words (GRID_PUT, an
    SPILL_N to a fixed word; the tables precede the spill slots) right after
    the last of them is defined, and each row is ``CHECK_GRID key, v_K`` with
    imm E_K and c = table word | (n - 1) << 10: j = E_K - key; j < n =>
    table[j] = v_K (mw_isa.h).  The row goes where the row's last check was.
    Same verdict as the checks, lane by lane: key = E_K - j holds for exactly
    the pair (K, k = j)."""
    groups: Dict[int, List[int]] = {}
    for i, ins in enumerate(insns):
        if ins.op == "CHECK_IMPEQK" and isinstance(ins.srcs[0], VReg):
            groups.setdefault(ins.srcs[0].id, []).append(i)
    defpos = {ins.dst.id: i for i, ins in enumerate(insns) if ins.dst is not None}
    nextid = 1 + max((v.id for ins in insns for v in ([ins.dst] if ins.dst is not None else []) + list(ins.srcs)
                      if isinstance(v, VReg)), default=-1)
    drop: set = set()
    after: Dict[int, List[MInsn]] = {}
    redrawn: set = set()
    t0 = 0
    for kid, pos in groups.items():
        if len(pos) < GRID_MIN:
            continue
        plan = _grid_plan(insns, pos)
        if plan is None:
            continue
        table, rows = plan
        n = len(table)
        if t0 + n > 1024:
            break
        key = insns[pos[0]].srcs[0]
        put = max([defpos[key.id]] + [defpos[t.id] for t in table if isinstance(t, VReg)])
        after.setdefault(put, []).extend(MInsn("GRID_PUT", 0, None, [t], imm=t0 + k) for k, t in enumerate(table))
        width = insns[pos[0]].width
        for r, (opnd, E, lastp) in rows.items():
            at = lastp if lastp > put else put
            d = insns[defpos[opnd.id]] if isinstance(opnd, VReg) else None
            if d is not None and d.op == "LEAF_N" and defpos[opnd.id] < put:
                # a leaf defined before the table: drawn again at its row rather
                # than kept live (a spill and a fill) across the program
                fresh = VReg(nextid, "N")
                nextid += 1
                after.setdefault(at, []).append(MInsn("LEAF_N", d.width, fresh, [], imm=d.imm))
                redrawn.add(opnd.id)
                opnd = fresh
            after.setdefault(at, []).append(MInsn("CHECK_GRID", width, None, [key, opnd, ("raw", t0 | (n - 1) << 10)],
                                                  imm=E))
        drop.update(pos)
        t0 += n
    if not drop:
        return insns
    out: List[MInsn] = []
    for i, ins in enumerate(insns):
        if i not in drop:
            out.append(ins)
        out.extend(after.get(i, ()))
    if redrawn:   # the leaves drawn again that nothing else reads any more
        uses = _uses(out)
        out = [ins for ins in out if not (ins.op == "LEAF_N" and ins.dst is not None and ins.dst.id in redrawn
                                          and not uses.get(ins.dst.id, 0))]
    return out


def _schedule_narrow_early(insns: List[MInsn]) -> List[MInsn]:
    """Move every instruction with a narrow (N) result right after the last
    definition of its operands.

    The operand-first order evaluates a conjunct's comparisons only when the
    conjunct's ``and`` tree is reached, so the wide values they read stay live
    across the rest of the chain (in C5, most of the spill traffic).  A
    narrow result costs one register, so evaluating it as soon as its operands
    exist never raises the wide live set and usually ends a wide operand's
    life.  CHECKs move with their operand too: a conjunct's comparisons are
    tested (and, with early exit, can stop the wave) as soon as they exist,
    instead of holding one register each until the conjunct's end.  Leaves (no
    operands) stay at their first use; STORE/END keep their place.
    """
    anchor: Dict[int, int] = {}           # vreg id -> index of the insn after which it is defined
    after: Dict[int, List[MInsn]] = {}    # original index -> hoisted insns emitted right after it
    head: List[MInsn] = []
    keep: List[bool] = []
    leafv = {ins.dst.id for ins in insns if ins.op.startswith("LEAF") and ins.dst is not None}
    for i, ins in enumerate(insns):
        # operands that are leaves do not count: leaves are defined at their first
        # use, often far above, and stay live anyway (hoisting to them would only
        # stretch the result's live range)
        srcs = [s for s in ins.srcs if isinstance(s, VReg)]
        nonleaf = any(s.id not in leafv for s in srcs)
        movable = ((ins.dst is not None and ins.dst.cls == "N" and nonleaf
                    and not ins.op.startswith(("LEAF", "FILL", "MOV")))
                   or (ins.op == "CHECK" and nonleaf))
        if movable and ins.op != "CHECK":
            # at most HOIST_CAP results per definition point: one wide value read
            # by thousands of comparisons (the congruence premises of a symbolic
            # calldata offset) would otherwise make them all live at once
            movable = len(after.get(max(anchor[s.id] for s in srcs), ())) < HOIST_CAP
        if movable:
            a = max(anchor[s.id] for s in srcs)
            after.setdefault(a, []).append(ins)
            if ins.dst is not None:
                anchor[ins.dst.id] = a
            keep.append(False)
        else:
            if ins.dst is not None:
                anchor[ins.dst.id] = i
            keep.append(True)
    out: List[MInsn] = list(head)
    for i, ins in enumerate(insns):
        if keep[i]:
            out.append(ins)
        out.extend(after.get(i, ()))
    return out


# --------------------------------------------------------------------------- register allocation
REMAT_LEAVES = os.environ.get("MYTHRIL_AMD_REMAT_LEAVES", "1") != "0"


def _allocate(insns: List[MInsn], slots: Optional[Tuple[int, int]] = None):
    """Belady allocation of W/N vregs to MW_NW/MW_NN slots (slots: fewer,
    (W, N) - mw_compile.cpp mw_compile_slots); returns (insns, n_spill)."""
    uses: Dict[int, List[int]] = {}
    for i, ins in enumerate(insns):
        for s in ins.srcs:
            if isinstance(s, VReg):
                uses.setdefault(s.id, []).append(i)
    ptr: Dict[int, int] = {k: 0 for k in uses}

    def next_use(vid: int, i: int) -> int:
        lst = uses.get(vid)
        if not lst:
            return 1 << 60
        p = ptr[vid]
        while p < len(lst) and lst[p] < i:
            p += 1
        ptr[vid] = p
        return lst[p] if p < len(lst) else 1 << 60

    nw, nn = slots or (isa.NW, isa.NN)
    # the interpreter's write-back scratch slots are never allocated (mw_isa.h)
    free = {"W": [k for k in range(nw - 1, -1, -1) if k != isa.W_RESERVED],
            "N": [k for k in range(nn - 1, -1, -1) if k & 31 != isa.N_RESERVED]}
    reg_of: Dict[int, int] = {}
    resident: Dict[str, Dict[int, VReg]] = {"W": {}, "N": {}}
    # spill slots: per class (a W slot is 8 words of the per-lane spill area,
    # an N slot 1 word); numbered here, laid out by _layout_spills
    spill_of: Dict[int, int] = {}
    spill_free: Dict[str, List[int]] = {"W": [], "N": []}
    slot_cls: List[str] = []
    out: List[MInsn] = []
    # wide leaves are drawn again where they are needed instead of spilled and
    # filled (REMAT_LEAVES): the candidate generator is a function of the
    # candidate and the leaf alone, and a W spill is eight words each way
    remat = {ins.dst.id: ins for ins in insns if ins.op == "LEAF_W" and ins.dst is not None} \
        if REMAT_LEAVES else {}
    rematted: set = set()

    def get_spill_slot(cls: str) -> int:
        if spill_free[cls]:
            return spill_free[cls].pop()
        slot_cls.append(cls)
        return len(slot_cls) - 1

    def evict(cls: str, i: int, pinned: set):
        best, best_nu = None, -1
        for vid, vr in resident[cls].items():
            if vid in pinned:
                continue
            nu = next_use(vid, i)
            if nu > best_nu:
                best, best_nu = vr, nu
        if best is None:
            raise Unsupported("register pressure: too many simultaneous operands")
        slot = reg_of.pop(best.id)
        del resident[cls][best.id]
        if best_nu < (1 << 60) and best.id in remat:
            rematted.add(best.id)
        elif best_nu < (1 << 60) and best.id not in spill_of:
            sp = get_spill_slot(cls)
            spill_of[best.id] = sp
            m = MInsn("SPILL_W" if cls == "W" else "SPILL_N", 0, None, [("phys", slot)], imm=sp)
            out.append(m)
        free[cls].append(slot)

    def take(cls: str, i: int, pinned: set) -> int:
        if not free[cls]:
            evict(cls, i, pinned)
        return free[cls].pop()

    for i, ins in enumerate(insns):
        pinned = {s.id for s in ins.srcs if isinstance(s, VReg)}
        # bring every source into a register
        for s in ins.srcs:
            if isinstance(s, VReg) and s.id not in reg_of:
                if s.id in rematted:
                    slot = take(s.cls, i, pinned)
                    r = remat[s.id]
                    out.append(MInsn("LEAF_W", r.width, ("phys", slot), [], r.imm, chain=r.chain))
                    reg_of[s.id] = slot
                    resident[s.cls][s.id] = s
                    continue
                if s.id not in spill_of:
                    raise AssertionError("use of undefined vreg")
                slot = take(s.cls, i, pinned)
                out.append(MInsn("FILL_W" if s.cls == "W" else "FILL_N", 0, ("phys", slot), [],
                                 imm=spill_of[s.id]))
                reg_of[s.id] = slot
                resident[s.cls][s.id] = s
        phys_srcs = []
        for s in ins.srcs:
            phys_srcs.append(("phys", reg_of[s.id]) if isinstance(s, VReg) else s)
        # release sources that die here (the interpreter reads before it writes)
        for s in ins.srcs:
            if isinstance(s, VReg) and s.id in reg_of and next_use(s.id, i + 1) >= (1 << 60):
                slot = reg_of.pop(s.id)
                resident[s.cls].pop(s.id, None)
                free[s.cls].append(slot)
                if s.id in spill_of:
                    spill_free[s.cls].append(spill_of.pop(s.id))
        dst = None
        if ins.dst is not None:
            d = ins.dst
            slot = take(d.cls, i, set())
            if next_use(d.id, i + 1) < (1 << 60):
                reg_of[d.id] = slot
                resident[d.cls][d.id] = d
            else:
                free[d.cls].append(slot)  # dead result (e.g. traced only) - slot reused
            dst = ("phys", slot)
        out.append(MInsn(ins.op, ins.width, dst, phys_srcs, ins.imm, chain=ins.chain))
    return _layout_spills(out, slot_cls)


def _layout_spills(insns: List[MInsn], slot_cls: List[str]):
    """Word offsets for the spill slots; returns (insns, spill words per lane).

    The first LDS_SPILL_WORDS words of a lane's spill area live in LDS and the
    rest in global memory (mw_kernels.hip), so slots are placed by traffic:
    most SPILL/FILL accesses per word first.  C3 (129 narrow slots) keeps its
    hottest 80 in LDS instead of the first 10 W-sized slots."""
    # the grid tables (_form_grids) come first, at the words their GRID_PUTs name
    tables = 1 + max((ins.imm for ins in insns if ins.op == "GRID_PUT"), default=-1)
    if not slot_cls:
        return insns, tables
    hits = [0] * len(slot_cls)
    for ins in insns:
        if ins.op in ("SPILL_W", "SPILL_N", "FILL_W", "FILL_N"):
            hits[ins.imm] += 1
    size = [8 if c == "W" else 1 for c in slot_cls]
    order = sorted(range(len(slot_cls)), key=lambda k: (-hits[k] / size[k], k))
    off, words = {}, tables
    for k in order:
        off[k] = words
        words += size[k]
    for ins in insns:
        if ins.op in ("SPILL_W", "SPILL_N", "FILL_W", "FILL_N"):
            ins.imm = off[ins.imm]
    return insns, words


LDS_SPILL_WORDS = 80   # mw_kernels.hip kLdsSpillWords


# --------------------------------------------------------------------------- encode
_POOL_RANDOM_W = (1).to_bytes(4, "little") + bytes(32)   # a RANDOM entry of a wide leaf


def _limbs(v: int) -> List[int]:
    return [(v >> (32 * k)) & 0xFFFFFFFF for k in range(8)]


def layout_leaves(leaf_nodes: Sequence[Node], leaf_specs: Optional[Dict[str, LeafSpec]] = None,
                  pools: Optional[Dict[str, List[Optional[int]]]] = None, memo: Optional[dict] = None):
    """Leaf table + pool words for `leaf_nodes` (in leaf-index order).

    Default layout: bit-interleaved (Morton) digits over the first
    INDEX_FIELD_BITS index bits, so every pool varies at small indices and the
    best proposals of all leaves are tried together first; leaves that do not
    fit are sampled with hashed digits.  Returns (specs, leaf words, pool
    words, input rows).  The code refers to leaves by index only, so a program
    whose leaf set grows (incremental.py) re-lays its table with this.
    memo: a long-lived context's pool bytes by (width, entries)."""
    specs: List[LeafSpec] = []
    leaf_words: List[int] = []
    pool_words = bytearray()   # u32 words, little-endian
    in_row = 0
    user = dict(leaf_specs or {})
    resolved: List[LeafSpec] = []
    for n in leaf_nodes:
        w = _w(n)
        spec = user.get(n.name)
        if spec is None and pools and n.name in pools:
            spec = LeafSpec(n.name, w, pool=list(pools[n.name]))
        if spec is None:
            spec = LeafSpec(n.name, w)
        spec.width = w
        if spec.pool:
            p = list(spec.pool)
            nb = max(0, math.ceil(math.log2(len(p)))) if len(p) > 1 else 0
            p += [None] * ((1 << nb) - len(p))
            spec.pool = p
        resolved.append(spec)
    by_name = {s.name: s for s in resolved}
    for spec in resolved:
        lead = by_name.get(spec.tie) if spec.tie else None
        if spec.tie and (lead is None or lead.tie or not lead.pool or not spec.pool
                         or len(lead.pool) != len(spec.pool)):
            spec.tie = None
    fresh = [s for s in resolved if s.pool and len(s.pool) > 1 and not s.hashed and s.bits == 0
             and s.shift == 0 and s.stride == 0 and not s.tie]
    if fresh:
        stride = len(fresh)
        for j, spec in enumerate(fresh):
            nb = int(math.log2(len(spec.pool)))
            top = j + (nb - 1) * stride
            if top < INDEX_FIELD_BITS:
                spec.bits, spec.shift, spec.stride = nb, j, stride
            else:
                fit = max(0, (INDEX_FIELD_BITS - 1 - j) // stride + 1)
                if fit >= 2:  # interleave the first 2^fit entries, hash nothing
                    spec.bits, spec.shift, spec.stride = fit, j, stride
                    spec.pool = spec.pool[:1 << fit]
                else:
                    spec.hashed = True
    for spec in resolved:
        if spec.tie:   # same digit as the leader: same layout, same hash key
            lead = by_name[spec.tie]
            spec.pool = spec.pool[:len(lead.pool)]
            spec.bits, spec.shift, spec.stride, spec.hashed = lead.bits, lead.shift, lead.stride, lead.hashed
            spec.salt = lead.key_salt()
    bit = 0
    for li, (n, spec) in enumerate(zip(leaf_nodes, resolved)):
        w = spec.width
        kind, pshift, pbits, poff, pstride = 0, 0, 0, 0, 0
        if spec.pool:
            nb = int(math.log2(len(spec.pool))) if len(spec.pool) > 1 else 0
            if spec.hashed:
                spec.bits, spec.shift, spec.stride = nb, 0, 0
                kind = 2
            elif spec.stride:
                kind = 3
            else:
                kind = 1
                if spec.bits == 0 and spec.shift == 0:
                    spec.bits = nb
            pshift, pbits, poff, pstride = spec.shift, spec.bits, len(pool_words) // 4, spec.stride
            bit = max(bit, spec.shift + (spec.bits - 1) * max(spec.stride, 1) + 1 if spec.bits else 0)
            key = (w, tuple(spec.pool)) if memo is not None else None
            pb = memo.get(key) if key is not None else None
            if pb is None:
                m = (1 << w) - 1
                if w < 32:   # one word per entry (mw_isa.h MW_POOL_NARROW_RANDOM)
                    pb = array("I", [isa.POOL_NARROW_RANDOM if e is None else e & m for e in spec.pool]).tobytes()
                else:        # flags word + 8 limbs, little-endian
                    pb = b"".join([_POOL_RANDOM_W if e is None else b"\0\0\0\0" + (e & m).to_bytes(32, "little")
                                   for e in spec.pool])
                if key is not None:
                    if len(memo) >= 1 << 16:
                        memo.clear()
                    memo[key] = pb
            pool_words += pb
        leaf_words.extend([w, kind, spec.key_salt(), pshift, pbits, poff, in_row, pstride])
        in_row += (w + 31) // 32
        specs.append(spec)
    if bit > 63:
        raise Unsupported("pool digit fields exceed the 64-bit candidate index")

    return specs, leaf_words, np.frombuffer(bytes(pool_words), dtype="<u4").astype(np.uint32), in_row


def compile_program(conjuncts: Sequence[Node], leaf_specs: Optional[Dict[str, LeafSpec]] = None,
                    trace: Sequence[Node] = (), pools: Optional[Dict[str, List[Optional[int]]]] = None,
                    slots: Optional[Tuple[int, int]] = None) -> Program:
    """Compile the conjunction of `conjuncts` (IR Bool terms).  slots: the
    (W, N) register slots the allocator may use, when fewer than MW_NW / MW_NN."""
    conj = _flatten(conjuncts)
    lw = _Lowerer()
    for t in trace:
        lw.trace_req[t.id] = t
    checks = 0
    for c in conj:
        lw.scope += 1
        if c.op == "const" and not c.val:
            lw.emit_void("CHECK", 1, [Const(0, "N")])
            checks += 1
            continue
        v = lw.lower(c)
        lw.emit_void("CHECK", 1, [v])
        checks += 1
    for t in trace:  # traced nodes not reachable from the conjuncts
        lw.lower(t)
    lw.emit_void("END", 0, [])

    lw.insns = _schedule_narrow_early(lw.insns)
    insns, n_spill = _allocate(_fuse_checks(lw.insns), slots)

    # constant pool
    consts: List[int] = []
    kmap: Dict[Tuple[int, str], int] = {}

    def kref(c: Const) -> int:
        key = (c.value, c.cls)
        if key not in kmap:
            kmap[key] = len(consts)
            consts.extend(_limbs(c.value) if c.cls == "W" else [c.value & 0xFFFFFFFF])
        return isa.KBIT | kmap[key]

    # trace rows
    trace_map: Dict[int, Tuple[int, str]] = {}
    rows = 0
    code: List[int] = []
    for k, ins in enumerate(insns):
        fields = []
        for s in ins.srcs:
            if isinstance(s, Const):
                fields.append(kref(s))
            else:
                fields.append(s[1])
        while len(fields) < 3:
            fields.append(0)
        imm = ins.imm
        if ins.op in ("STORE_W", "STORE_N"):
            nid = -imm - 1
            cls = "W" if ins.op == "STORE_W" else "N"
            trace_map[nid] = (rows, cls)
            imm = rows
            rows += 8 if cls == "W" else 1
        dcls = isa.SHAPES[ins.op][0] if ins.dst is not None else None
        dst = isa.encode_dst(dcls, ins.dst[1] if ins.dst is not None else 0)
        # the chain holds only if the consumer still follows directly (no FILL/SPILL/STORE between)
        nxt = insns[k + 1] if k + 1 < len(insns) else None
        flags = isa.FLAG_CHAIN if (ins.chain and nxt is not None and nxt.op == "W_CDINS" and nxt.srcs
                                   and nxt.srcs[0] == ins.dst) else 0
        op = "SPILL_N" if ins.op == "GRID_PUT" else ins.op
        code.extend(isa.encode(op, ins.width, dst, fields[0], fields[1], fields[2], imm, flags))
    if len(consts) > 0x7FFF:
        raise Unsupported("constant pool overflow")

    specs, leaf_words, pool_words, in_row = layout_leaves(lw.leaf_nodes, leaf_specs, pools)

    reach = topo(conj + list(trace))
    ops = sum(node_cost(n) for n in reach)
    # wide divisions: their nominal price (without the signed ops' 4L sign
    # handling, which always runs) is replaced by the executed path's price in
    # Program.executed_ops
    div_nominal_ops, n_div = 0, 0
    for n in reach:
        if n.op in ("bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod") and _w(n) > isa.NARROW_MAX:
            L = (_w(n) + 31) // 32
            div_nominal_ops += node_cost(n) - (4 * L if n.op in ("bvsdiv", "bvsrem", "bvsmod") else 0)
            n_div += 1
    arr = lambda x: np.asarray(x if x else [0], dtype=np.uint32)
    stats = {"nodes": len(reach), "insns": len(code) // 4, "spills": sum(1 for i in insns if i.op.startswith("SPILL")),
             "fills": sum(1 for i in insns if i.op.startswith("FILL")),
             "div_nominal_ops": div_nominal_ops, "wide_divisions": n_div}
    return Program(code=np.asarray(code, dtype=np.uint32), consts=arr(consts),
                   leaves=np.asarray(leaf_words, dtype=np.uint32),
                   pool=pool_words if pool_words.size else arr([]),
                   n_spill=n_spill, n_trace_rows=rows, n_input_rows=in_row, ops_per_eval=ops,
                   leaf_specs=specs, leaf_nodes=list(lw.leaf_nodes), trace_map=trace_map,
                   n_insn=len(code) // 4, n_conjuncts=checks, stats=stats, ssa=list(lw.insns))
