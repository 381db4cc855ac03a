"""IR -> IR preprocessing before bytecode compilation.

1. **Arrays** (``mythril/laser/smt/array.py:168-227``: ``N_calldata`` 256->8,
   ``balance`` 256->256, ``Storage`` arrays, ``K`` constant arrays):
   ``select`` over ``store`` chains is unfolded into ``ite`` chains
   (``select(store(A,i,v),j) = ite(i=j, v, select(A,j))``), ``select(K(v),j) = v``,
   ``select(ite(c,A,B),j) = ite(c, select(A,j), select(B,j))``.  Every remaining
   base read ``select(A, j)`` becomes a fresh leaf (**Ackermannisation**):
   named ``A@<hex>`` for a concrete index (so the same cell is the same leaf in
   every program), ``A@s<k>`` otherwise.
2. **Uninterpreted functions** (``mythril/laser/smt/function.py``; the keccak
   UFs ``keccak256_N`` / ``keccak256_N-1`` of
   ``keccak_function_manager.py:71-84``, ``Power`` of
   ``exponent_function_manager.py:22``) are treated the same way: one leaf per
   distinct application.
3. **Congruence**: for every pair of reads of one array / applications of one
   function whose indices/arguments are not both concrete,
   ``(args_t = args_u) => (val_t = val_u)`` is added as a conjunct, so any
   satisfying assignment of the leaves extends to a model of the arrays/UFs.
4. **Width legalisation**: equalities over terms wider than 256 bits (512-bit
   keccak inputs from ``Concat`` in ``instructions.py:1016-1030``,
   ``bitvec.py:79-85`` zero-padded ``==``) are split into 256-bit chunks, and
   extracts are pushed through ``concat`` / ``zero_extend`` / ``extract``.
   Anything that still needs >256-bit arithmetic raises ``Unsupported``.

The result records, per synthesized leaf, which array/function cell it stands
for (:class:`AckLeaf`) so a witness can be turned back into a model.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from .compiler import Unsupported
from .ir import BOOL, Ctx, Node, topo

MAXW = 256


@dataclass
class AckLeaf:
    name: str
    kind: str             # "select" | "apply"
    base: str             # array or function name
    args: Tuple[Node, ...]  # index term(s) in the rewritten formula
    width: int
    value: Optional[Node] = None  # defined (not free) value: keccak inverse = the hashed input


@dataclass
class Lowered:
    conjuncts: List[Node]
    ack: Dict[str, AckLeaf] = field(default_factory=dict)
    congruence: int = 0


class _Rewriter:
    def __init__(self, ctx: Ctx):
        self.ctx = ctx
        self.memo: Dict[int, Node] = {}
        self.ack: Dict[str, AckLeaf] = {}
        self.by_base: Dict[str, List[AckLeaf]] = {}
        self.leaf_of_key: Dict[tuple, Node] = {}
        self.inner_apply: Dict[int, tuple] = {}   # leaf id of f(x) -> (f, x)
        self.nsym = 0

    # -- extract simplification (pushes extracts towards leaves) ------------------
    def extract(self, x: Node, hi: int, lo: int) -> Node:
        c = self.ctx
        if lo == 0 and hi == x.width - 1:
            return x
        if x.op == "const":
            return c.const(x.val >> lo, hi - lo + 1)
        if x.op == "extract":
            return self.extract(x.args[0], hi + x.params[1], lo + x.params[1])
        if x.op == "zero_extend":
            inner = x.args[0]
            if lo >= inner.width:
                return c.const(0, hi - lo + 1)
            if hi < inner.width:
                return self.extract(inner, hi, lo)
            part = self.extract(inner, inner.width - 1, lo)
            return c.app("zero_extend", part, params=(hi - inner.width + 1,))
        if x.op == "concat":
            parts = []
            off = x.width
            pieces = []
            for a in x.args:
                off -= a.width
                pieces.append((a, off))  # a occupies [off, off + a.width)
            for a, aoff in pieces:
                ahi = aoff + a.width - 1
                if ahi < lo or aoff > hi:
                    continue
                parts.append(self.extract(a, min(hi, ahi) - aoff, max(lo, aoff) - aoff))
            return parts[0] if len(parts) == 1 else c.app("concat", *parts)
        if x.width > MAXW:
            raise Unsupported(f"extract from a {x.width}-bit {x.op}")
        return c.app("extract", x, params=(hi, lo))

    def chunks(self, x: Node) -> List[Node]:
        """x as 256-bit (or narrower, last) chunks, least significant first."""
        out = []
        lo = 0
        while lo < x.width:
            hi = min(x.width, lo + MAXW) - 1
            out.append(self.extract(x, hi, lo))
            lo = hi + 1
        return out

    def eq(self, a: Node, b: Node) -> Node:
        c = self.ctx
        if a.width <= MAXW:
            return c.app("=", a, b)
        parts = [c.app("=", x, y) for x, y in zip(self.chunks(a), self.chunks(b))]
        return c.app("and", *parts) if len(parts) > 1 else parts[0]

    # -- leaves for array reads / UF applications ---------------------------------
    def _key_name(self, base: str, args: Tuple[Node, ...]) -> Tuple[tuple, str]:
        if all(a.op == "const" for a in args):
            key = (base,) + tuple((a.width, a.val) for a in args)
            nm = f"{base}@" + ",".join(f"{a.val:x}" for a in args)
        else:
            key = (base,) + tuple(("t", a.id) for a in args)
            self.nsym += 1
            nm = f"{base}@s{self.nsym}"
        return key, nm

    def read_leaf(self, kind: str, base: str, args: Tuple[Node, ...], width: int) -> Node:
        key, nm = self._key_name(base, args)
        leaf = self.leaf_of_key.get(key)
        if leaf is None:
            leaf = self.wide_var(nm, width)
            self.leaf_of_key[key] = leaf
            al = AckLeaf(nm, kind, base, args, width)
            self.ack[nm] = al
            self.by_base.setdefault((kind, base), []).append(al)
        return leaf

    def defined_leaf(self, base: str, args: Tuple[Node, ...], width: int, value: Node) -> Node:
        """An application whose value is a term (no free leaf); still congruence-checked."""
        key = ("def", base) + tuple(("t", a.id) for a in args)
        if key not in self.leaf_of_key:
            self.nsym += 1
            nm = f"{base}@d{self.nsym}"
            al = AckLeaf(nm, "apply", base, args, width, value=value)
            self.ack[nm] = al
            self.by_base.setdefault(("apply", base), []).append(al)
            self.leaf_of_key[key] = value
        return self.leaf_of_key[key]

    def wide_var(self, nm: str, width: int) -> Node:
        """A leaf; wider than 256 bits it is the concat of 256-bit chunk leaves nm#0 (LSB).."""
        if width <= MAXW:
            return self.ctx.var(nm, width)
        parts = []
        lo, k = 0, 0
        while lo < width:
            cw = min(MAXW, width - lo)
            parts.append(self.ctx.var(f"{nm}#{k}", cw))
            lo += cw
            k += 1
        return self.ctx.app("concat", *parts[::-1])

    def select(self, arr: Node, idx: Node) -> Node:
        c = self.ctx
        # walk store chains / ite / K
        if arr.op == "array":
            return self.read_leaf("select", arr.name, (idx,), arr.width)
        if arr.op == "const_array":
            return arr.args[0]
        if arr.op == "store":
            base, i, v = arr.args
            if i.op == "const" and idx.op == "const":
                return v if i.val == idx.val else self.select(base, idx)
            return c.app("ite", self.eq(i, idx), v, self.select(base, idx))
        if arr.op == "ite":
            cond, a1, a2 = arr.args
            return c.app("ite", cond, self.select(a1, idx), self.select(a2, idx))
        raise Unsupported(f"select from {arr.op}")

    # -- main rewrite --------------------------------------------------------------
    def rw(self, root: Node) -> Node:
        for n in topo([root]):
            if n.id in self.memo:
                continue
            self.memo[n.id] = self._rw1(n)
        return self.memo[root.id]

    def _rw1(self, n: Node) -> Node:
        c = self.ctx
        if n.op == "const":
            return n
        if n.op == "var":
            return self.wide_var(n.name, n.width) if n.width > MAXW else n
        if n.op == "array":
            return n  # only reachable through select/store, handled there
        args = [self.memo[a.id] for a in n.args]
        op = n.op
        if op == "select":
            return self.select(args[0], args[1])
        if op in ("store", "const_array"):
            return c._mk(op, n.width, tuple(args), n.params, n.val, n.name, n.dom)
        if op == "ite" and n.is_array:
            return c._mk("ite", n.width, tuple(args), dom=n.dom)
        if op == "apply":
            # Mythril's keccak inverse (keccak_function_manager.py:80-81): inv(keccak256_N(x)) is
            # *defined* as x.  Sound: every inverse application sits on a keccak application
            # here, and the inverse congruence (k_t = k_u) => (x_t = x_u) is still emitted, so
            # any witness extends to a model with inv(k_t) = x_t (the condition
            # inv(func(x)) == x of :169-179 then holds by construction).
            if n.name.endswith("-1") and len(args) == 1:
                inner = self.inner_apply.get(args[0].id)
                if inner is not None and inner[0] == n.name[:-2] and inner[1].width == n.width:
                    return self.defined_leaf(n.name, (args[0],), n.width, inner[1])
            leaf = self.read_leaf("apply", n.name, tuple(args), n.width)
            if len(args) == 1:
                self.inner_apply[leaf.id] = (n.name, args[0])
            return leaf
        if op in ("=", "distinct") and args and args[0].is_array:
            raise Unsupported("array equality")
        if op == "=" and args[0].width > MAXW:
            eqs = [self.eq(args[0], b) for b in args[1:]]
            return c.app("and", *eqs) if len(eqs) > 1 else eqs[0]
        if op == "distinct" and args[0].width > MAXW:
            if len(args) != 2:
                raise Unsupported("wide n-ary distinct")
            return c.app("not", self.eq(args[0], args[1]))
        if op == "extract":
            return self.extract(args[0], n.params[0], n.params[1])
        if op in ("concat", "zero_extend") and n.width > MAXW:
            # kept only as an operand of a wide =, which chunks it via extract
            return c._mk(op, n.width, tuple(args), n.params)
        return c.app(op, *args, params=n.params) if op not in ("ite",) else c.app("ite", *args)

    def congruence(self) -> List[Node]:
        c = self.ctx
        out = []
        for (kind, base), reads in self.by_base.items():
            for t, u in _pair_order(reads):
                    if all(a.op == "const" for a in t.args) and all(a.op == "const" for a in u.args):
                        continue  # distinct concrete cells: nothing to relate
                    if any(_never_equal(x, y) for x, y in zip(t.args, u.args)):
                        continue  # e.g. cells base+3 and base+7 of one symbolic offset
                    same = [self.eq(*_fold_offsets(c, x, y)) for x, y in zip(t.args, u.args)]
                    prem = c.app("and", *same) if len(same) > 1 else same[0]
                    vt = t.value if t.value is not None else self.wide_var(t.name, t.width)
                    vu = u.value if u.value is not None else self.wide_var(u.name, u.width)
                    out.append(c.app("=>", prem, self.eq(vt, vu)))
        return out


def _offset(n: Node):
    """(base, k) with n == base + k (mod 2^w), for a const k; (n, 0) otherwise."""
    if n.op == "bvadd" and len(n.args) == 2:
        a, b = n.args
        if b.op == "const" and a.op != "const":
            return a, b.val
        if a.op == "const" and b.op != "const":
            return b, a.val
    return n, 0


PAIR_TILE = 12   # symbolic cells kept resident while the concrete cells stream past


def _pair_order(reads):
    """Every unordered pair of one array's/function's reads, ordered for the
    register file: symbolic-symbolic pairs first, then the concrete x symbolic
    pairs in tiles of PAIR_TILE symbolic reads.  Within a tile each concrete
    cell is used PAIR_TILE times in a row and the tile's symbolic cells stay
    in registers, instead of the narrow file refilling one of 32+ live cells at
    every pair (C3: 2 371 -> ~300 fills)."""
    sym = [r for r in reads if not all(a.op == "const" for a in r.args)]
    con = [r for r in reads if all(a.op == "const" for a in r.args)]
    out = [(sym[i], sym[j]) for i in range(len(sym)) for j in range(i + 1, len(sym))]
    for k in range(0, len(sym), PAIR_TILE):
        tile = sym[k:k + PAIR_TILE]
        out += [(c, s) for c in con for s in tile]
    return out


def _fold_offsets(c: Ctx, x: Node, y: Node):
    """x = y with a constant offset moved across: (b + k = K) -> (b = K - k), so
    every congruence premise of one symbolic calldata offset compares the SAME
    base term with constants (one live value instead of one per cell)."""
    for a, k in ((x, y), (y, x)):
        if k.op == "const":
            b, off = _offset(a)
            if off and b.width == a.width:
                return b, c.const(k.val - off, a.width)
    return x, y


def _never_equal(x: Node, y: Node) -> bool:
    """True when x = y is false under every assignment: two distinct constants,
    or one term plus two different constant offsets (the bytes of one ABI word
    read at a symbolic calldata offset, calldata.py:218-231)."""
    if x.op == "const" and y.op == "const":
        return x.val != y.val
    (bx, kx), (by, ky) = _offset(x), _offset(y)
    return bx is by and x.width == y.width and (kx - ky) % (1 << x.width) != 0


def lower_constraints(conjuncts: List[Node], ctx: Ctx) -> Lowered:
    rw = _Rewriter(ctx)
    out = [rw.rw(cj) for cj in conjuncts]
    cong = rw.congruence()
    for n in topo(out + cong):
        if n.width > MAXW and n.op not in ("concat", "zero_extend", "var"):
            raise Unsupported(f"{n.op} on {n.width} bits")
        if n.op in ("concat", "zero_extend") and n.width > MAXW:
            raise Unsupported(f"{n.width}-bit {n.op} outside an equality")
    return Lowered(out + cong, rw.ack, len(cong))


def needs_lowering(conjuncts: List[Node]) -> bool:
    for n in topo(conjuncts):
        if n.op in ("select", "apply", "store", "const_array", "array") or n.width > MAXW:
            return True
    return False
