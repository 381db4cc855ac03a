"""A stand-in for the z3 Python module over our IR (TEST INFRASTRUCTURE).

z3 is not installable here or on the GPU box, so the z3 half
of the drop-in is exercised against this: ASTs with ``get_id`` / ``eq`` /
``children`` / ``decl().kind()`` / ``params`` / sorts / numerals as z3py
exposes them, one AST object per distinct term (z3 hash-conses its ASTs), and
a ``Solver`` whose ``sexpr()`` prints with our SMT-LIB printer.  The kind
numbers are arbitrary; the walker looks them up by name, as it does in z3.
Parity with the real z3 API stays unpinned."""
from __future__ import annotations

import types

from mythril_amd.ir import BOOL
from mythril_amd.smt2 import to_smt2

_NAMES = ["Z3_OP_TRUE", "Z3_OP_FALSE", "Z3_OP_EQ", "Z3_OP_DISTINCT", "Z3_OP_ITE", "Z3_OP_AND", "Z3_OP_OR",
          "Z3_OP_IFF", "Z3_OP_XOR", "Z3_OP_NOT", "Z3_OP_IMPLIES", "Z3_OP_BNUM", "Z3_OP_BNEG", "Z3_OP_BADD",
          "Z3_OP_BSUB", "Z3_OP_BMUL", "Z3_OP_BSDIV", "Z3_OP_BUDIV", "Z3_OP_BSREM", "Z3_OP_BUREM", "Z3_OP_BSMOD",
          "Z3_OP_BSDIV_I", "Z3_OP_BUDIV_I", "Z3_OP_BSREM_I", "Z3_OP_BUREM_I", "Z3_OP_BSMOD_I", "Z3_OP_ULEQ",
          "Z3_OP_SLEQ", "Z3_OP_UGEQ", "Z3_OP_SGEQ", "Z3_OP_ULT", "Z3_OP_SLT", "Z3_OP_UGT", "Z3_OP_SGT",
          "Z3_OP_BAND", "Z3_OP_BOR", "Z3_OP_BNOT", "Z3_OP_BXOR", "Z3_OP_BNAND", "Z3_OP_BNOR", "Z3_OP_BXNOR",
          "Z3_OP_CONCAT", "Z3_OP_SIGN_EXT", "Z3_OP_ZERO_EXT", "Z3_OP_EXTRACT", "Z3_OP_REPEAT", "Z3_OP_BREDOR",
          "Z3_OP_BREDAND", "Z3_OP_BCOMP", "Z3_OP_BSHL", "Z3_OP_BLSHR", "Z3_OP_BASHR", "Z3_OP_ROTATE_LEFT",
          "Z3_OP_ROTATE_RIGHT", "Z3_OP_BUMUL_NO_OVFL", "Z3_OP_BSMUL_NO_OVFL", "Z3_OP_BSMUL_NO_UDFL",
          "Z3_OP_SELECT", "Z3_OP_STORE", "Z3_OP_CONST_ARRAY", "Z3_OP_UNINTERPRETED"]
KIND = {n: 0x100 + i for i, n in enumerate(_NAMES)}
# IR op -> the kind z3 gives the term (independent of mythril_amd/z3walk.py's table)
_OF_OP = {"=": "Z3_OP_EQ", "distinct": "Z3_OP_DISTINCT", "ite": "Z3_OP_ITE", "and": "Z3_OP_AND",
          "or": "Z3_OP_OR", "xor": "Z3_OP_XOR", "not": "Z3_OP_NOT", "=>": "Z3_OP_IMPLIES",
          "bvneg": "Z3_OP_BNEG", "bvadd": "Z3_OP_BADD", "bvsub": "Z3_OP_BSUB", "bvmul": "Z3_OP_BMUL",
          "bvsdiv": "Z3_OP_BSDIV", "bvudiv": "Z3_OP_BUDIV", "bvsrem": "Z3_OP_BSREM", "bvurem": "Z3_OP_BUREM",
          "bvsmod": "Z3_OP_BSMOD", "bvule": "Z3_OP_ULEQ", "bvsle": "Z3_OP_SLEQ", "bvuge": "Z3_OP_UGEQ",
          "bvsge": "Z3_OP_SGEQ", "bvult": "Z3_OP_ULT", "bvslt": "Z3_OP_SLT", "bvugt": "Z3_OP_UGT",
          "bvsgt": "Z3_OP_SGT", "bvand": "Z3_OP_BAND", "bvor": "Z3_OP_BOR", "bvnot": "Z3_OP_BNOT",
          "bvxor": "Z3_OP_BXOR", "bvnand": "Z3_OP_BNAND", "bvnor": "Z3_OP_BNOR", "bvxnor": "Z3_OP_BXNOR",
          "concat": "Z3_OP_CONCAT", "sign_extend": "Z3_OP_SIGN_EXT", "zero_extend": "Z3_OP_ZERO_EXT",
          "extract": "Z3_OP_EXTRACT", "repeat": "Z3_OP_REPEAT", "bvcomp": "Z3_OP_BCOMP", "bvshl": "Z3_OP_BSHL",
          "bvlshr": "Z3_OP_BLSHR", "bvashr": "Z3_OP_BASHR", "rotate_left": "Z3_OP_ROTATE_LEFT",
          "rotate_right": "Z3_OP_ROTATE_RIGHT", "bvumul_noovfl": "Z3_OP_BUMUL_NO_OVFL",
          "bvsmul_noovfl": "Z3_OP_BSMUL_NO_OVFL", "bvsmul_noudfl": "Z3_OP_BSMUL_NO_UDFL",
          "select": "Z3_OP_SELECT", "store": "Z3_OP_STORE", "const_array": "Z3_OP_CONST_ARRAY",
          "var": "Z3_OP_UNINTERPRETED", "array": "Z3_OP_UNINTERPRETED", "apply": "Z3_OP_UNINTERPRETED"}
S_BOOL, S_BV, S_ARRAY = 1, 4, 5


class Sort:
    def __init__(self, kind, size=0, dom=None, rng=None):
        self._k, self._s, self._d, self._r = kind, size, dom, rng

    def kind(self):
        return self._k

    def size(self):
        return self._s

    def domain(self):
        return self._d

    def range(self):
        return self._r


def _sort_of(n) -> Sort:
    if n.is_array:
        return Sort(S_ARRAY, dom=Sort(S_BV, n.dom), rng=Sort(S_BV, n.width))
    return Sort(S_BOOL) if n.width == BOOL else Sort(S_BV, n.width)


class Decl:
    def __init__(self, n):
        self.n = n

    def kind(self):
        n = self.n
        if n.op == "const":
            return KIND["Z3_OP_BNUM"] if n.width != BOOL else KIND["Z3_OP_TRUE" if n.val else "Z3_OP_FALSE"]
        return KIND[_OF_OP[n.op]]

    def name(self):
        return self.n.name if self.n.name is not None else self.n.op

    def params(self):
        return list(self.n.params) if self.n.op != "apply" else []

    def arity(self):
        return len(self.n.args)

    def domain(self, i):
        return Sort(S_BV, self.n.params[i])

    def range(self):
        return Sort(S_BV, self.n.width)


class Ast:
    """One z3 AST: an IR node seen through z3py's interface."""
    __slots__ = ("node", "z")

    def __init__(self, node, z):
        self.node, self.z = node, z

    def get_id(self):
        return self.node.id

    def eq(self, other):
        return isinstance(other, Ast) and other.node is self.node

    def children(self):
        return [self.z.ast(a) for a in self.node.args]

    def num_args(self):
        return len(self.node.args)

    def decl(self):
        return Decl(self.node)

    def sort(self):
        return _sort_of(self.node)

    def as_long(self):
        return self.node.val

    def size(self):
        return self.node.width


def module(name: str = "z3") -> types.ModuleType:
    """A fresh stand-in module: ``ast(node)`` gives the (shared) AST of an IR node."""
    z = types.ModuleType(name)
    for k, v in KIND.items():
        setattr(z, k, v)
    z.Z3_BOOL_SORT, z.Z3_BV_SORT, z.Z3_ARRAY_SORT = S_BOOL, S_BV, S_ARRAY
    table = {}
    z.calls = {"sexpr": 0, "children": 0}

    def ast(node):
        a = table.get(id(node))          # the node itself (ids repeat across contexts); Ast keeps it alive
        if a is None:
            a = table[id(node)] = Ast(node, z)
        return a
    z.ast = ast

    class Solver:
        def __init__(self):
            self.items = []

        def add(self, items):
            self.items.extend(items if isinstance(items, list) else [items])

        def sexpr(self):
            z.calls["sexpr"] += 1
            return to_smt2([a.node for a in self.items])
    z.Solver = Solver
    return z
