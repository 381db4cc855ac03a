"""z3 AST -> IR without printing.

The text route (z3bridge: ``Solver.sexpr()`` then our SMT-LIB parser) costs
in proportion to the size of every new conjunct's TEXT: a JUMPI condition on
a calldata word prints the word's 32 guarded byte reads again (~6 KB), although
z3 shares that subterm with every earlier conjunct.  This walker reads the
z3 AST itself - ``decl().kind()``, ``children()``, ``params()``, sorts and
numerals - and memoises every translated AST by id (kept alive, confirmed with
``eq``: z3 reuses the ids of collected ASTs).  A new conjunct then costs only
its new nodes; the shared subterms are one dictionary lookup each.

It produces exactly the terms the text route produces (the same IR ops,
widths, parameters and names; tests/test_z3walk.py checks both routes give
byte-identical programs).  Anything it does not know - an operator kind, a
sort - raises ``Unsupported`` and the caller uses the text route, which fails
closed to the reference solver in turn.

Operator kinds are looked up by name in the z3 module (``Z3_OP_*``), so a z3
build that lacks one simply leaves it unmapped.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Tuple

from .compiler import Unsupported
from .ir import BOOL, Ctx, Node
from .smt2 import Decl, Sort


class SortConflict(Unsupported):
    """One symbol name met with two sorts (z3 allows it; one IR context cannot hold both)."""

# z3 operator kind name -> IR op (SMT-LIB names; the _I division variants as
# the parser's ALIASES read them)
_OPS = {
    "Z3_OP_EQ": "=", "Z3_OP_DISTINCT": "distinct", "Z3_OP_ITE": "ite", "Z3_OP_AND": "and", "Z3_OP_OR": "or",
    "Z3_OP_IFF": "=", "Z3_OP_XOR": "xor", "Z3_OP_NOT": "not", "Z3_OP_IMPLIES": "=>",
    "Z3_OP_BNEG": "bvneg", "Z3_OP_BADD": "bvadd", "Z3_OP_BSUB": "bvsub", "Z3_OP_BMUL": "bvmul",
    "Z3_OP_BSDIV": "bvsdiv", "Z3_OP_BUDIV": "bvudiv", "Z3_OP_BSREM": "bvsrem", "Z3_OP_BUREM": "bvurem",
    "Z3_OP_BSMOD": "bvsmod", "Z3_OP_BSDIV_I": "bvsdiv", "Z3_OP_BUDIV_I": "bvudiv", "Z3_OP_BSREM_I": "bvsrem",
    "Z3_OP_BUREM_I": "bvurem", "Z3_OP_BSMOD_I": "bvsmod",
    "Z3_OP_ULEQ": "bvule", "Z3_OP_SLEQ": "bvsle", "Z3_OP_UGEQ": "bvuge", "Z3_OP_SGEQ": "bvsge",
    "Z3_OP_ULT": "bvult", "Z3_OP_SLT": "bvslt", "Z3_OP_UGT": "bvugt", "Z3_OP_SGT": "bvsgt",
    "Z3_OP_BAND": "bvand", "Z3_OP_BOR": "bvor", "Z3_OP_BNOT": "bvnot", "Z3_OP_BXOR": "bvxor",
    "Z3_OP_BNAND": "bvnand", "Z3_OP_BNOR": "bvnor", "Z3_OP_BXNOR": "bvxnor", "Z3_OP_CONCAT": "concat",
    "Z3_OP_BCOMP": "bvcomp", "Z3_OP_BSHL": "bvshl", "Z3_OP_BLSHR": "bvlshr", "Z3_OP_BASHR": "bvashr",
    "Z3_OP_BUMUL_NO_OVFL": "bvumul_noovfl", "Z3_OP_BSMUL_NO_OVFL": "bvsmul_noovfl",
    "Z3_OP_BSMUL_NO_UDFL": "bvsmul_noudfl",
    "Z3_OP_SELECT": "select", "Z3_OP_STORE": "store",
}
# indexed operators: the IR op and how many integer parameters it takes
_INDEXED = {"Z3_OP_EXTRACT": ("extract", 2), "Z3_OP_ZERO_EXT": ("zero_extend", 1),
            "Z3_OP_SIGN_EXT": ("sign_extend", 1), "Z3_OP_REPEAT": ("repeat", 1),
            "Z3_OP_ROTATE_LEFT": ("rotate_left", 1), "Z3_OP_ROTATE_RIGHT": ("rotate_right", 1)}


class Z3Walker:
    """Translates z3 expressions into one IR context, memoised per AST."""

    def __init__(self, z3, ctx: Ctx):
        self.z3 = z3
        self.ctx = ctx
        self.memo: Dict[int, Tuple[object, Node]] = {}   # AST id -> (AST kept alive, IR node)
        self.decls: Dict[str, Decl] = {}
        k = {}
        for name, op in _OPS.items():
            v = getattr(z3, name, None)
            if v is not None:
                k[v] = op
        self.kinds = k
        self.indexed = {getattr(z3, n): spec for n, spec in _INDEXED.items() if getattr(z3, n, None) is not None}
        self.K_UNINT = getattr(z3, "Z3_OP_UNINTERPRETED", None)
        self.K_TRUE, self.K_FALSE = getattr(z3, "Z3_OP_TRUE", None), getattr(z3, "Z3_OP_FALSE", None)
        self.K_BNUM = getattr(z3, "Z3_OP_BNUM", None)
        self.K_CONST_ARRAY = getattr(z3, "Z3_OP_CONST_ARRAY", None)
        self.K_REDOR, self.K_REDAND = getattr(z3, "Z3_OP_BREDOR", None), getattr(z3, "Z3_OP_BREDAND", None)
        self.S_BOOL, self.S_BV = getattr(z3, "Z3_BOOL_SORT", None), getattr(z3, "Z3_BV_SORT", None)
        self.S_ARRAY = getattr(z3, "Z3_ARRAY_SORT", None)

    def _sort(self, s) -> Sort:
        k = s.kind()
        if k == self.S_BOOL:
            return Sort("bool")
        if k == self.S_BV:
            return Sort("bv", s.size())
        if k == self.S_ARRAY:
            d, r = self._sort(s.domain()), self._sort(s.range())
            if d.kind != "bv" or r.kind != "bv":
                raise Unsupported("z3walk: only bitvector arrays")
            return Sort("array", r.width, d.width)
        raise Unsupported(f"z3walk: sort kind {k}")

    def _declare(self, name: str, args: List[Sort], sort: Sort) -> None:
        old = self.decls.get(name)
        if old is None:
            self.decls[name] = Decl(name, args, sort)
        elif old.sort != sort or old.args != args:
            raise SortConflict(f"z3walk: {name} declared with two sorts")

    def term(self, root) -> Node:
        """The IR term of one z3 expression (operands first, iteratively)."""
        memo = self.memo
        rid = root.get_id()
        hit = memo.get(rid)
        if hit is not None and (hit[0] is root or hit[0].eq(root)):
            return hit[1]
        stack = [(root, rid, None)]
        while stack:
            e, eid, kids = stack[-1]
            if kids is None:
                hit = memo.get(eid)
                if hit is not None and (hit[0] is e or hit[0].eq(e)):
                    stack.pop()
                    continue
                kids = [(c, c.get_id()) for c in e.children()]
                stack[-1] = (e, eid, kids)
                pending = False
                for c, cid in reversed(kids):
                    h = memo.get(cid)
                    if h is None or not (h[0] is c or h[0].eq(c)):
                        stack.append((c, cid, None))
                        pending = True
                if pending:
                    continue
            stack.pop()
            memo[eid] = (e, self._node(e, [memo[cid][1] for _, cid in kids]))
        return memo[rid][1]

    def _node(self, e, args: List[Node]) -> Node:
        c = self.ctx
        d = e.decl()
        k = d.kind()
        op = self.kinds.get(k)
        if op is not None:
            return c.app(op, *args)
        if not args:
            if k == self.K_TRUE:
                return c.true()
            if k == self.K_FALSE:
                return c.false()
            if k == self.K_BNUM:
                return c.const(e.as_long(), e.size())
            if k == self.K_UNINT:
                name = d.name()
                srt = self._sort(e.sort())
                self._declare(name, [], srt)
                if srt.kind == "bool":
                    return c.var(name, BOOL)
                if srt.kind == "bv":
                    return c.var(name, srt.width)
                return c.array(name, srt.dom, srt.width)
            raise Unsupported(f"z3walk: constant of kind {k}")
        spec = self.indexed.get(k)
        if spec is not None:
            ps = [int(p) for p in d.params()]
            if len(ps) != spec[1]:
                raise Unsupported(f"z3walk: {spec[0]} with parameters {ps}")
            return c.app(spec[0], *args, params=ps)
        if k == self.K_UNINT:
            name = d.name()
            self._declare(name, [self._sort(d.domain(i)) for i in range(d.arity())], self._sort(d.range()))
            rng = self.decls[name].sort
            if rng.kind != "bv":
                raise Unsupported(f"z3walk: function {name} of sort {rng.kind}")
            return c.apply(name, rng.width, *args)
        if k == self.K_CONST_ARRAY:
            srt = self._sort(e.sort())
            return c.const_array(srt.dom, args[0])
        if k == self.K_REDOR or k == self.K_REDAND:
            (x,) = args
            ones = k == self.K_REDAND
            eq = c.app("=", x, c.const(-1 if ones else 0, x.width))
            return c.app("ite", eq, c.const(1 if ones else 0, 1), c.const(0 if ones else 1, 1))
        raise Unsupported(f"z3walk: operator {d.name()} (kind {k})")


def available(z3) -> bool:
    """The z3 module has what the walker reads (every z3py release does)."""
    return all(getattr(z3, n, None) is not None for n in ("Z3_OP_UNINTERPRETED", "Z3_OP_BNUM", "Z3_BV_SORT"))
