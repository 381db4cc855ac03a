"""Constraint DAG IR: hash-consed bitvector / bool / array terms.

This is the data structure both the front ends (SMT-LIB2 text, z3 ASTs) produce
and the compiler consumes.  It models exactly the term vocabulary Mythril's
path constraints are built from:

* ``mythril/laser/smt/bitvec.py:126-309``      BitVec operators (+ - * / & | ^ < > <= >= == != << >>)
* ``mythril/laser/smt/bitvec_helper.py:30-242`` LShR/If/UGT/ULT/UGE/ULE/Concat/Extract/URem/SRem/UDiv/Sum/
  BVAddNoOverflow/BVMulNoOverflow/BVSubNoUnderflow
* ``mythril/laser/smt/bool.py:340-376``         And/Or/Xor/Not
* ``mythril/laser/smt/array.py:168-227``        Array/K select/store
* ``mythril/laser/smt/function.py:7-29``        uninterpreted function application

plus the forms z3's ``simplify`` rewrites them into (n-ary add/mul/and/or,
``bvnot``, ``bvumul_noovfl``, the ``*_i`` division variants, ``=>``...).

Op names are SMT-LIB 2.6 names.  Widths: ``w >= 1`` for bitvectors, ``0`` for
Bool.  Array terms carry ``dom``/``rng`` widths (``width`` == ``rng``).
"""
from __future__ import annotations

from typing import Dict, Iterable, List, Optional, Sequence, Tuple

BOOL = 0

# ops whose result is Bool
BOOL_OPS = frozenset({
    "and", "or", "not", "xor", "=>", "=", "distinct",
    "bvult", "bvule", "bvugt", "bvuge", "bvslt", "bvsle", "bvsgt", "bvsge",
    "bvumul_noovfl", "bvsmul_noovfl", "bvsmul_noudfl",
    "bvaddc",   # internal: carry out of a w-bit add (wide-arithmetic legalisation, lower.py)
})

# bitvector ops: name -> (min arity, max arity or None for n-ary)
BV_OPS = {
    "bvadd": (1, None), "bvmul": (1, None), "bvand": (1, None), "bvor": (1, None),
    "bvxor": (1, None), "concat": (1, None),
    "bvsub": (2, 2), "bvudiv": (2, 2), "bvurem": (2, 2), "bvsdiv": (2, 2),
    "bvsrem": (2, 2), "bvsmod": (2, 2), "bvshl": (2, 2), "bvlshr": (2, 2),
    "bvashr": (2, 2), "bvnand": (2, 2), "bvnor": (2, 2), "bvxnor": (2, 2),
    "bvcomp": (2, 2),
    "bvneg": (1, 1), "bvnot": (1, 1),
    "extract": (1, 1), "zero_extend": (1, 1), "sign_extend": (1, 1),
    "repeat": (1, 1), "rotate_left": (1, 1), "rotate_right": (1, 1),
}

# z3-internal spellings that mean the same thing once the divisor is known
# non-zero (z3 wraps them in ``ite (= y 0) ...``); we give them the SMT-LIB
# total semantics, which agrees wherever z3's value is specified.
ALIASES = {
    "bvudiv_i": "bvudiv", "bvurem_i": "bvurem", "bvsdiv_i": "bvsdiv",
    "bvsrem_i": "bvsrem", "bvsmod_i": "bvsmod",
}

LEAF_OPS = frozenset({"const", "var", "array", "apply_leaf"})


class Node:
    """One hash-consed term.  Never construct directly; use :class:`Ctx`."""

    __slots__ = ("op", "width", "args", "params", "val", "name", "dom", "id", "_h")

    def __init__(self, op, width, args, params, val, name, dom, nid, h=None):
        self.op = op
        self.width = width
        self.args = args
        self.params = params
        self.val = val
        self.name = name
        self.dom = dom
        self.id = nid
        self._h = h   # computed on first use (__hash__): most terms are never hashed

    # -- sort helpers -------------------------------------------------
    @property
    def is_bool(self) -> bool:
        return self.width == BOOL and self.dom is None

    @property
    def is_array(self) -> bool:
        return self.dom is not None

    def __hash__(self):
        h = self._h
        if h is None:
            h = self._h = hash((self.op, self.width, tuple(a.id for a in self.args), self.params, self.val,
                                self.name, self.dom))
        return h

    def __repr__(self):  # pragma: no cover - debugging aid
        if self.op == "const":
            return f"#{self.val:x}[{self.width}]" if self.width else ("true" if self.val else "false")
        if self.op in ("var", "array"):
            return f"{self.name}"
        inner = " ".join(repr(a) for a in self.args)
        p = "".join(f" {x}" for x in self.params)
        n = f" {self.name}" if self.name else ""
        return f"({self.op}{p}{n} {inner})"


class Ctx:
    """Term factory with structural hash-consing (same term -> same Node)."""

    def __init__(self):
        self._tab: Dict[tuple, Node] = {}
        self.nodes: List[Node] = []

    def _mk(self, op, width, args=(), params=(), val=None, name=None, dom=None) -> Node:
        if params.__class__ is not tuple:
            params = tuple(params)
        na = len(args)
        if na == 2:
            a, b = args
            ids = (a.id, b.id)
        elif na == 1:
            ids = (args[0].id,)
        else:
            ids = tuple([a.id for a in args])
        key = (op, width, ids, params, val, name, dom)
        n = self._tab.get(key)
        if n is None:
            n = Node(op, width, args if args.__class__ is tuple else tuple(args), params, val, name, dom,
                     len(self.nodes))
            self._tab[key] = n
            self.nodes.append(n)
        return n

    # -- leaves -------------------------------------------------------
    def const(self, val: int, width: int) -> Node:
        if width == BOOL:
            return self._mk("const", BOOL, val=1 if val else 0)
        return self._mk("const", width, val=val & ((1 << width) - 1))

    def true(self) -> Node:
        return self.const(1, BOOL)

    def false(self) -> Node:
        return self.const(0, BOOL)

    def var(self, name: str, width: int) -> Node:
        return self._mk("var", width, name=name)

    def array(self, name: str, dom: int, rng: int) -> Node:
        return self._mk("array", rng, name=name, dom=dom)

    def const_array(self, dom: int, value: Node) -> Node:
        return self._mk("const_array", value.width, (value,), dom=dom)

    # -- generic application -------------------------------------------
    def app(self, op: str, *args: Node, params: Sequence[int] = ()) -> Node:
        op = ALIASES.get(op, op)
        params = tuple(int(p) for p in params)
        if op == "=>" and len(args) > 2:
            # SMT-LIB: => is right-associative, (=> a b c) = (=> a (=> b c))
            acc = args[-1]
            for a in reversed(args[:-1]):
                acc = self._mk("=>", BOOL, (a, acc))
            return acc
        if op in BOOL_OPS:
            return self._mk(op, BOOL, args, params)
        if op == "ite":
            c, a, b = args
            if a.is_array:
                return self._mk("ite", a.width, args, dom=a.dom)
            return self._mk("ite", a.width, args)
        if op == "select":
            arr, idx = args
            return self._mk("select", arr.width, args)
        if op == "store":
            arr, idx, v = args
            return self._mk("store", arr.width, args, dom=arr.dom)
        if op not in BV_OPS:
            raise KeyError(f"unsupported op {op!r}")
        w = bv_result_width(op, [a.width for a in args], params)
        return self._mk(op, w, args, params)

    def apply(self, fname: str, rng: int, *args: Node) -> Node:
        """Uninterpreted function application ``fname(args) : (_ BitVec rng)``."""
        return self._mk("apply", rng, args, params=tuple(a.width for a in args), name=fname)


def bv_result_width(op: str, ws: Sequence[int], params: Sequence[int]) -> int:
    if op == "concat":
        return sum(ws)
    if op == "extract":
        hi, lo = params
        if not (0 <= lo <= hi < ws[0]):
            raise ValueError(f"bad extract {hi},{lo} of width {ws[0]}")
        return hi - lo + 1
    if op in ("zero_extend", "sign_extend"):
        return ws[0] + params[0]
    if op == "repeat":
        return ws[0] * params[0]
    if op == "bvcomp":
        return 1
    w = ws[0]
    for x in ws[1:]:
        if x != w:
            raise ValueError(f"width mismatch in {op}: {ws}")
    return w


def topo(roots: Iterable[Node], seen: Optional[set] = None) -> List[Node]:
    """Post-order (operands first) list of every node reachable from roots.
    `seen` (optional, updated in place): ids already visited by an earlier
    call; those nodes and everything under them are skipped."""
    out: List[Node] = []
    if seen is None:
        seen = set()
    emit, mark = out.append, seen.add
    for r in roots:
        if r.id in seen:
            continue
        stack: List[Node] = [r]
        push, pop = stack.append, stack.pop
        while stack:
            n = stack[-1]
            if n.id in seen:
                pop()
                continue
            pending = False
            for a in reversed(n.args):   # first operand on top: the same order as a recursive walk
                if a.id not in seen:
                    push(a)
                    pending = True
            if not pending:
                pop()
                mark(n.id)
                emit(n)
    return out


def free_vars(roots: Iterable[Node]) -> List[Node]:
    return [n for n in topo(roots) if n.op in ("var", "array") or n.op == "apply"]
