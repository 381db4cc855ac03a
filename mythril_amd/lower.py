"""IR -> IR preprocessing before bytecode compilation.

1. **Arrays** (``mythril/laser/smt/array.py:168-227``: ``N_calldata`` 256->8,
   ``balance`` 256->256, ``Storage`` arrays, ``K`` constant arrays):
   ``select`` over ``store`` chains is unfolded into ``ite`` chains
   (``select(store(A,i,v),j) = ite(i=j, v, select(A,j))``), ``select(K(v),j) = v``,
   ``select(ite(c,A,B),j) = ite(c, select(A,j), select(B,j))``.  Every remaining
   base read ``select(A, j)`` becomes a fresh leaf (**Ackermannisation**):
   named ``A@<hex>`` for a concrete index (so the same cell is the same leaf in
   every program), ``A@s<h>`` otherwise, ``h`` a structural hash of the index
   term (not its position in the query: a conjunct lowers to the same terms
   in every set that holds it, which lets ``lower_constraints`` reuse a
   conjunct's lowering across queries).
2. **Uninterpreted functions** (``mythril/laser/smt/function.py``; the keccak
   UFs ``keccak256_N`` / ``keccak256_N-1`` of
   ``keccak_function_manager.py:71-84``, ``Power`` of
   ``exponent_function_manager.py:22``) are treated the same way: one leaf per
   distinct application.
3. **Congruence**: for every pair of reads of one array / applications of one
   function whose indices/arguments are not both concrete,
   ``(args_t = args_u) => (val_t = val_u)`` is added as a conjunct, so any
   satisfying assignment of the leaves extends to a model of the arrays/UFs.
4. **Width legalisation** (generic in the width): every term wider than 256
   bits is decomposed into 256-bit chunks (least significant first) when a
   narrower term consumes it:
   * structure (``concat``, ``extract``, ``zero_extend``, ``sign_extend``,
     ``repeat``, rotates and shifts by constants) regroups bit slices;
   * ``bvand/bvor/bvxor/bvnot`` and ``ite`` work chunk by chunk;
   * ``bvadd/bvsub/bvneg`` propagate carries between chunks with the
     carry-out op ``bvaddc`` (``N_ADDC``), e.g. ``BVAddNoOverflow``'s 257-bit
     add (``bitvec_helper.py:196-208``, z3 ``Z3_mk_bvadd_no_overflow``:
     ``extract(256,256, zext1 a + zext1 b) = 0``, SWC-101 ``integer.py:143``)
     becomes ``not(bvaddc(a, b))``;
   * ``=``/``distinct`` compare chunks; unsigned/signed orderings compare
     chunks lexicographically from the top (sign bit flipped for signed);
   * 512-bit keccak inputs (``instructions.py:1016-1030``) and the
     zero-padded ``==`` of ``bitvec.py:79-85`` are the same mechanism.
   Wide ``bvmul``/division/remainder and shifts by a non-constant amount still
   raise ``Unsupported`` (fail closed to z3).

The result records, per synthesized leaf, which array/function cell it stands
for (:class:`AckLeaf`) so a witness can be turned back into a model.
"""
from __future__ import annotations

import zlib
from itertools import chain
from dataclasses import dataclass, field
from operator import attrgetter
from typing import Dict, List, Optional, Tuple

from . import isa
from .compiler import Unsupported, _flatten
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
    flat: List[Node] = field(default_factory=list)    # conjuncts with top-level `and` flattened, `true` dropped
    nodes: List[Node] = field(default_factory=list)   # topo(flat): every node the search program evaluates
    # what harvest reads (the congruence premises unkeyed, _Rewriter.keyed): None = conjuncts / nodes
    harvest_conjuncts: Optional[List[Node]] = None
    harvest_nodes: Optional[List[Node]] = None
    # long-lived contexts: (length of the main conjuncts' part of the harvest
    # nodes, the congruence part's node ids) - harvest keeps its scan of that
    # part, identical while a set's reads are (pools.harvest segments)
    harvest_split: Optional[Tuple[int, tuple]] = None


class _Rewriter:
    def __init__(self, ctx: Ctx):
        self.ctx = ctx
        self.memo: Dict[int, Node] = {}
        self.ack: Dict[str, AckLeaf] = {}
        self.by_base: Dict[str, List[AckLeaf]] = {}
        self.leaf_of_key: Dict[tuple, Node] = {}
        self.inner_apply: Dict[int, tuple] = {}   # leaf id of f(x) -> (f, x)
        self.seg_memo: Dict[int, List[Node]] = {}
        self.chunk_memo: Dict[int, List[Node]] = {}
        # leaves a top-level conjunct fixes (leaf = K): the congruence reads K
        # in their place (equivalent under that conjunct, candidate by candidate)
        self.pins: Dict[str, Node] = {}

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
            return self._assemble(self._slice(self.segs(x), lo, hi))
        return c.app("extract", x, params=(hi, lo))

    # -- wide terms as 256-bit chunks ------------------------------------------------
    def chunks(self, x: Node) -> List[Node]:
        """x as 256-bit (or narrower, last) chunks, least significant first."""
        if x.width <= MAXW:
            return [x]
        got = self.chunk_memo.get(x.id)
        if got is None:
            segs = self.segs(x)
            got = []
            lo = 0
            while lo < x.width:
                hi = min(x.width, lo + MAXW) - 1
                got.append(self._assemble(self._slice(segs, lo, hi)))
                lo = hi + 1
            self.chunk_memo[x.id] = got
        return got

    def _slice(self, segs: List[Node], lo: int, hi: int) -> List[Node]:
        """Bits [lo, hi] of an LSB-first slice list, as LSB-first slices."""
        c = self.ctx
        out: List[Node] = []
        off = 0
        for t in segs:
            a, b = max(lo, off), min(hi, off + t.width - 1)
            if a <= b:
                if a == off and b == off + t.width - 1:
                    out.append(t)
                else:
                    out.append(self.extract(t, b - off, a - off))
            off += t.width
        return out

    def _assemble(self, segs: List[Node]) -> Node:
        """One term (<= 256 bits) from LSB-first slices."""
        if len(segs) == 1:
            return segs[0]
        if all(t.op == "const" for t in segs):
            v, off = 0, 0
            for t in segs:
                v |= t.val << off
                off += t.width
            return self.ctx.const(v, off)
        return self.ctx.app("concat", *segs[::-1])

    def segs(self, x: Node) -> List[Node]:
        """x as LSB-first slices of at most 256 bits each (any boundaries)."""
        if x.width <= MAXW:
            return [x]
        got = self.seg_memo.get(x.id)
        if got is None:
            got = self._segs(x)
            assert sum(t.width for t in got) == x.width, (x.op, x.width)
            self.seg_memo[x.id] = got
        return got

    def _segs(self, x: Node) -> List[Node]:
        c = self.ctx
        op, w = x.op, x.width
        if op == "const":
            return [c.const(x.val >> lo, min(MAXW, w - lo)) for lo in range(0, w, MAXW)]
        if op == "var":
            return [c.var(f"{x.name}#{k}", min(MAXW, w - lo)) for k, lo in enumerate(range(0, w, MAXW))]
        if op == "concat":
            out: List[Node] = []
            for a in reversed(x.args):
                out.extend(self.segs(a))
            return out
        if op == "zero_extend":
            return self.segs(x.args[0]) + _zeros(c, x.params[0])
        if op == "sign_extend":
            a = x.args[0]
            sbit = self.extract(a, a.width - 1, a.width - 1)
            neg = c.app("=", sbit, c.const(1, 1))
            fill = []
            n = x.params[0]
            while n:
                k = min(MAXW, n)
                fill.append(c.app("ite", neg, c.const((1 << k) - 1, k), c.const(0, k)))
                n -= k
            return self.segs(a) + fill
        if op == "extract":
            hi, lo = x.params
            return self._slice(self.segs(x.args[0]), lo, hi)
        if op == "repeat":
            return self.segs(x.args[0]) * x.params[0]
        if op in ("rotate_left", "rotate_right"):
            r = x.params[0] % w
            if op == "rotate_right":
                r = (w - r) % w
            if r == 0:
                return self.segs(x.args[0])
            sg = self.segs(x.args[0])
            return self._slice(sg, w - r, w - 1) + self._slice(sg, 0, w - r - 1)   # (x << r) | (x >> (w - r))
        if op in ("bvshl", "bvlshr", "bvashr"):
            a, amt = x.args
            if amt.op != "const":
                raise Unsupported(f"{w}-bit {op} by a variable amount")
            k = amt.val
            sg = self.segs(a)
            if op == "bvshl":
                return _zeros(c, w) if k >= w else _zeros(c, k) + self._slice(sg, 0, w - k - 1)
            if op == "bvlshr":
                return _zeros(c, w) if k >= w else self._slice(sg, k, w - 1) + _zeros(c, k)
            k = min(k, w)
            top = self._slice(sg, w - 1, w - 1)[0]
            neg = c.app("=", top, c.const(1, 1))
            fill = []
            n = k
            while n:
                m = min(MAXW, n)
                fill.append(c.app("ite", neg, c.const((1 << m) - 1, m), c.const(0, m)))
                n -= m
            return (self._slice(sg, k, w - 1) if k < w else []) + fill
        # element-wise and arithmetic ops: on aligned 256-bit chunks
        if op == "ite":
            cond, a, b = x.args
            return [c.app("ite", cond, p, q) for p, q in zip(self.chunks(a), self.chunks(b))]
        if op in ("bvand", "bvor", "bvxor"):
            cols = zip(*[self.chunks(a) for a in x.args])
            return [c.app(op, *col) for col in cols]
        if op in ("bvnot", "bvnand", "bvnor", "bvxnor"):
            if op == "bvnot":
                return [c.app("bvnot", p) for p in self.chunks(x.args[0])]
            inner = {"bvnand": "bvand", "bvnor": "bvor", "bvxnor": "bvxor"}[op]
            return [c.app("bvnot", c.app(inner, p, q)) for p, q in zip(self.chunks(x.args[0]), self.chunks(x.args[1]))]
        if op == "bvadd":
            acc = self.chunks(x.args[0])
            for b in x.args[1:]:
                acc = self._add_chunks(acc, self.chunks(b), None)
            return acc
        if op == "bvsub":
            nb = [c.app("bvnot", q) for q in self.chunks(x.args[1])]
            return self._add_chunks(self.chunks(x.args[0]), nb, c.true())
        if op == "bvneg":
            nb = [c.app("bvnot", q) for q in self.chunks(x.args[0])]
            return self._add_chunks([c.const(0, q.width) for q in nb], nb, c.true())
        raise Unsupported(f"{op} on {w} bits")

    def _add_chunks(self, A: List[Node], B: List[Node], cin: Optional[Node]) -> List[Node]:
        """Chunk-wise a + b (+ cin), carries through bvaddc; folds zero operands."""
        c = self.ctx
        out = []
        carry = cin
        for a, b in zip(A, B):
            w = a.width
            if a.op == "const" and a.val == 0:
                a, b = b, a
            if b.op == "const" and b.val == 0:
                s, co = a, None
            else:
                s, co = c.app("bvadd", a, b), c.app("bvaddc", a, b)
            if carry is not None and not (carry.op == "const" and not carry.val):
                one = c.const(1, w) if carry.op == "const" else c.app("ite", carry, c.const(1, w), c.const(0, w))
                if s.op == "const" and s.val == 0:
                    s2, co2 = one, None
                else:
                    s2, co2 = c.app("bvadd", s, one), c.app("bvaddc", s, one)
                s = s2
                co = co2 if co is None else (co if co2 is None else c.app("or", co, co2))
            out.append(s)
            carry = co
        return out

    def eq(self, a: Node, b: Node) -> Node:
        c = self.ctx
        if a.width <= MAXW:
            return c.app("=", a, b)
        parts = [c.app("=", x, y) for x, y in zip(self.chunks(a), self.chunks(b))]
        return c.app("and", *parts) if len(parts) > 1 else parts[0]

    def ult(self, a: Node, b: Node, signed: bool) -> Node:
        """a < b on chunks, lexicographic from the most significant chunk."""
        c = self.ctx
        A, B = self.chunks(a), self.chunks(b)
        if signed:   # flip the sign bit, compare unsigned
            tw = A[-1].width
            m = c.const(1 << (tw - 1), tw)
            A = A[:-1] + [c.app("bvxor", A[-1], m)]
            B = B[:-1] + [c.app("bvxor", B[-1], m)]
        lt = None
        for p, q in zip(A, B):
            here = c.app("bvult", p, q)
            lt = here if lt is None else c.app("or", here, c.app("and", c.app("=", p, q), lt))
        return lt

    # -- leaves for array reads / UF applications ---------------------------------
    def _key_name(self, base: str, args: Tuple[Node, ...]) -> Tuple[tuple, str]:
        if len(args) == 1 and args[0].op == "const":   # a cell at a concrete index (calldata bytes)
            a = args[0]
            return (base, (a.width, a.val)), f"{base}@{a.val:x}"
        if all(a.op == "const" for a in args):
            key = (base,) + tuple((a.width, a.val) for a in args)
            nm = f"{base}@" + ",".join(f"{a.val:x}" for a in args)
        else:
            key = (base,) + tuple(("t", a.id) for a in args)
            nm = self._unique_name(f"{base}@s{_shash_args(self.ctx, args):016x}", args)
        return key, nm

    def _unique_name(self, nm: str, args: Tuple[Node, ...]) -> str:
        """nm for these argument terms, made unique in the context: a 64-bit
        structural hash that collides for two different argument tuples gets a
        suffix, so two reads never merge into one leaf (the context
        is hash-consed, so equal terms have equal ids)."""
        names = self.ctx.__dict__.setdefault("_ack_names", {})
        ids, base, k = tuple(a.id for a in args), nm, 0
        while names.setdefault(nm, ids) != ids:
            k += 1
            nm = f"{base}~{k}"
        return nm

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
            nm = self._unique_name(f"{base}@d{_shash_args(self.ctx, args):016x}", args)
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
        """The rewrite of root: operands first, each node once per rewriter
        (the walk of ir.topo with the memo as its visited set, so _rw1 runs in
        topo order: leaf names and congruence pairs do not depend on it)."""
        memo = self.memo
        got = memo.get(root.id)
        if got is not None:
            return got
        rw1 = self._rw1
        stack = [root]
        push, pop = stack.append, stack.pop
        while stack:
            n = stack[-1]
            if n.id in memo:
                pop()
                continue
            pending = False
            for a in reversed(n.args):
                if a.id not in memo:
                    push(a)
                    pending = True
            if not pending:
                pop()
                op = n.op
                # constants, arrays and leaves up to 256 bits rewrite to themselves (_rw1)
                memo[n.id] = n if (op == "const" or op == "array" or (op == "var" and n.width <= MAXW)) else rw1(n)
        return memo[root.id]

    def _rw1(self, n: Node) -> Node:
        c = self.ctx
        if n.op == "const":
            return n
        if n.op == "var":
            return self.wide_var(n.name, n.width) if n.width > MAXW else n
        if n.op == "array":
            return n  # only reachable through select/store, handled there
        memo = self.memo
        args = [memo[a.id] for a in n.args]
        op = n.op
        # unchanged operands and nothing to rewrite at this node: hash-consing
        # would return n itself (most nodes of a LASER query)
        if (op not in _REWRITE and n.width <= MAXW and n.dom is None and tuple(args) == n.args
                and (op not in _WIDE_ARG_OPS or max(map(_width, args)) <= MAXW)):
            return n
        if op == "select":
            return self.select(args[0], args[1])
        if op in ("store", "const_array"):
            return c._mk(op, n.width, tuple(args), n.params, n.val, n.name, n.dom)
        if op == "ite" and n.is_array:
            return c._mk("ite", n.width, tuple(args), dom=n.dom)
        if op in _POW2_OPS and len(args) == 2 and n.width <= MAXW:
            r = self._pow2(op, args, n.width)
            if r is not None:
                return r
        if op in ("=", "not") and n.width == BOOL:
            r = self._bool_bv(op, args)
            if r is not None:
                return r
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
        wide_args = bool(args) and max(map(_width, args)) > MAXW and any(
            a.width > MAXW and not a.is_array for a in args)
        if op == "=" and wide_args:
            eqs = [self.eq(args[0], b) for b in args[1:]]
            return c.app("and", *eqs) if len(eqs) > 1 else eqs[0]
        if op == "distinct" and wide_args:
            ne = [c.app("not", self.eq(args[i], args[j]))
                  for i in range(len(args)) for j in range(i + 1, len(args))]
            return c.app("and", *ne) if len(ne) > 1 else ne[0]
        if op == "bvcomp" and wide_args:
            return c.app("ite", self.eq(args[0], args[1]), c.const(1, 1), c.const(0, 1))
        if op in _ORDER and wide_args:
            name, swap, strict = _ORDER[op]
            a, b = (args[1], args[0]) if swap else (args[0], args[1])
            signed = name == "s"
            if strict:
                return self.ult(a, b, signed)
            return c.app("not", self.ult(b, a, signed))
        if op == "extract":
            return self.extract(args[0], n.params[0], n.params[1])
        if n.width > MAXW or wide_args:
            # a wide term is kept as built; whatever narrower term consumes it
            # decomposes it into chunks (extract / eq / ult above)
            if op in ("bvmul", "bvudiv", "bvurem", "bvsdiv", "bvsrem", "bvsmod", "bvumul_noovfl",
                      "bvsmul_noovfl", "bvsmul_noudfl"):
                raise Unsupported(f"{op} on {max(a.width for a in args)} bits")
            return c._mk(op, n.width, tuple(args), n.params)
        # what c.app(op, *args, params=n.params) builds: every rewrite keeps its
        # node's width, so the result width is n's
        return c._mk(op, n.width, tuple(args), n.params)

    def _pow2(self, op: str, args: List[Node], w: int) -> Optional[Node]:
        """z3 ``simplify`` rewrites (bv_rewriter) that turn arithmetic by a power
        of two into structure: ``x / 2^k``, ``x >> k`` -> ``concat(0, extract)``;
        ``x % 2^k``, ``x & (2^k - 1)`` -> ``concat(0, extract)``;
        ``x * 2^k``, ``x << k`` -> ``concat(extract, 0)``.  Solidity's selector
        dispatch ``div(calldataload(0), 2^224) & 0xffffffff`` then reaches the
        calldata bytes as an extract, which the candidate pools project through,
        and the kernels run no division for it."""
        c = self.ctx
        x, k = args
        if op in ("bvmul", "bvand") and x.op == "const" and k.op != "const":
            x, k = k, x
        if k.op != "const":
            return None
        v = k.val
        if op == "bvand":
            if v == 0:
                return c.const(0, w)
            if v & (v + 1):        # not of the form 2^j - 1
                return None
            j = v.bit_length()
            return x if j >= w else c.app("concat", c.const(0, w - j), self.extract(x, j - 1, 0))
        if op in ("bvshl", "bvlshr"):
            j = v
        else:
            if v == 0 or v & (v - 1):
                return None
            j = v.bit_length() - 1
        if op in ("bvudiv", "bvlshr"):
            if j == 0:
                return x
            return c.const(0, w) if j >= w else c.app("concat", c.const(0, j), self.extract(x, w - 1, j))
        if op == "bvurem":
            return c.const(0, w) if j == 0 else (x if j >= w else
                                                 c.app("concat", c.const(0, w - j), self.extract(x, j - 1, 0)))
        # bvmul, bvshl
        if j == 0:
            return x
        return c.const(0, w) if j >= w else c.app("concat", self.extract(x, w - 1 - j, 0), c.const(0, j))

    def _bool_bv(self, op: str, args: List[Node]) -> Optional[Node]:
        """z3 ``simplify``'s folding of EVM's Bool-as-word round trips
        (``util.pop_bitvec``'s ``If(b, 1, 0)``, ISZERO, JUMPI's ``cond != 0``):
        ``If(c, K1, K2) = K`` -> ``c`` / ``not c`` / a constant, ``not not c`` -> ``c``.
        The comparison inside then reaches the candidate pools' domains
        (e.g. ``call_value = 0`` from a non-payable check)."""
        c = self.ctx
        if op == "not":
            x = args[0]
            if x.op == "not":
                return x.args[0]
            if x.op == "const":
                return c.const(0 if x.val else 1, BOOL)
            return None
        if len(args) != 2:
            return None
        a, b = args
        if a.op == "const" and b.op != "const":
            a, b = b, a
        if b.op != "const" or a.op != "ite" or a.width == BOOL:
            return None
        cond, k1, k2 = a.args
        if k1.op != "const" or k2.op != "const":
            return None
        t1, t2 = k1.val == b.val, k2.val == b.val
        if t1 and t2:
            return c.true()
        if not t1 and not t2:
            return c.false()
        return cond if t1 else (cond.args[0] if cond.op == "not" else c.app("not", cond))

    def congruence(self, memo: Optional[dict] = None) -> List[Node]:
        """memo: the pairs' conjuncts kept with a long-lived context (a pair of
        reads is the same pair, by leaf name, in every set that holds both)."""
        c = self.ctx
        out = []
        for (kind, base), reads in self.by_base.items():
            for t, u in _pair_order(reads):
                if memo is not None:
                    pt, pu = self.pins.get(t.name), self.pins.get(u.name)
                    key = (t.name, u.name) if pt is None and pu is None else \
                        (t.name, u.name, pt and pt.val, pu and pu.val)
                    got = memo.get(key, 0)
                    if got != 0:
                        if got is not None:
                            out.append(got)
                        continue
                r = self._pair(t, u)
                if memo is not None:
                    memo[key] = r
                if r is not None:
                    out.append(r)
        return out

    def keyed(self, cong: List[Node], memo: Optional[dict] = None) -> List[Node]:
        """The congruence conjuncts with their index premises keyed: a wide
        index against a constant (base = K - k, the bytes of an ABI word at
        a symbolic calldata offset) becomes a 32-bit compare of the base's
        index key with K - k + KEY_BIAS (_index_key), for bases with at least
        KEY_MIN such premises (single-argument pairs of narrow values,
        _narrow_imp): one narrow term per base instead of a wide compare per
        diagonal of the pair grid, which compiler._fuse_checks folds into the
        check itself (CHECK_IMPEQK), so no premise flag stays live across the
        grid.  The harvest reads the unkeyed conjuncts.
        memo (a long-lived context's): per conjunct id, (base, K) or None and
        its keyed form - the same in every set whose count keys that base."""
        shapes = [self._shape(n, memo) for n in cong]
        count: Dict[int, int] = {}
        for sh in shapes:
            if sh is not None:
                bid = sh[0].id
                count[bid] = count.get(bid, 0) + 1
        if not count or max(count.values()) < KEY_MIN:
            return cong
        c = self.ctx
        out = []
        for n, sh in zip(cong, shapes):
            if sh is not None and count[sh[0].id] >= KEY_MIN:
                got = memo.get(("k", n.id)) if memo is not None else None
                if got is None:
                    got = self._keyed_imp(n, sh)
                    if memo is not None:
                        memo[("k", n.id)] = got
                n = got
            out.append(n)
        return out

    def _shape(self, n: Node, memo: Optional[dict]):
        if memo is not None:
            got = memo.get(n.id, 0)
            if got != 0:
                return got
        sh = _wide_index_eq(n.args[0]) if _narrow_imp(n) else None
        if memo is not None:
            memo[n.id] = sh
        return sh

    def _keyed_imp(self, n: Node, sh) -> Node:
        b, k = sh
        v = (k + KEY_BIAS) & ((1 << b.width) - 1)
        if v >= KEY_LIMIT:
            return n
        c = self.ctx
        return c.app("=>", c.app("=", self._index_key(b), c.const(v, 32)), n.args[1])

    def _index_key(self, b: Node) -> Node:
        """ite(hi(b + KEY_BIAS) = 0, lo32(b + KEY_BIAS), 0xffffffff): for
        e < KEY_LIMIT, key = e holds exactly when b = e - KEY_BIAS (mod 2^w)
        (e never equals the all-ones sentinel); the bias covers K < k too."""
        key = self.__dict__.setdefault("_keys", {})
        got = key.get(b.id)
        if got is None:
            c, w = self.ctx, b.width
            s = c.app("bvadd", b, c.const(KEY_BIAS, w))
            got = c.app("ite", c.app("=", self.extract(s, w - 1, 32), c.const(0, w - 32)),
                        self.extract(s, 31, 0), c.const(0xFFFFFFFF, 32))
            key[b.id] = got
        return got

    def _value(self, t: AckLeaf) -> Node:
        if t.value is not None:
            return t.value
        pin = self.pins.get(t.name)
        return pin if pin is not None else self.wide_var(t.name, t.width)

    def _pair(self, t: AckLeaf, u: AckLeaf) -> Optional[Node]:
        c = self.ctx
        if all(a.op == "const" for a in t.args) and all(a.op == "const" for a in u.args):
            return None   # distinct concrete cells: nothing to relate
        if any(_never_equal(x, y) for x, y in zip(t.args, u.args)):
            return None   # e.g. cells base+3 and base+7 of one symbolic offset
        # an argument both reads share (Power(256, k) and Power(256, i): the same
        # constant node) adds nothing to the premise
        same = [self.eq(*_fold_offsets(c, x, y)) for x, y in zip(t.args, u.args) if x is not y]
        vt, vu = self._value(t), self._value(u)
        if not same:
            return self.eq(vt, vu)
        prem = c.app("and", *same) if len(same) > 1 else same[0]
        return c.app("=>", prem, self.eq(vt, vu))


_POW2_OPS = frozenset({"bvudiv", "bvurem", "bvmul", "bvand", "bvshl", "bvlshr"})
# ops _rw1 may rewrite even when their operands are unchanged
_REWRITE = _POW2_OPS | {"select", "store", "const_array", "apply", "extract", "=", "not", "distinct", "bvcomp"}
# narrow results that may read wide operands (every other op's result is as wide as its operands)
_WIDE_ARG_OPS = frozenset({"bvult", "bvugt", "bvule", "bvuge", "bvslt", "bvsgt", "bvsle", "bvsge",
                           "bvumul_noovfl", "bvsmul_noovfl", "bvsmul_noudfl", "bvaddc"})
_width = attrgetter("width")

# wide orderings: op -> (signedness, swap operands, strict)
_ORDER = {"bvult": ("u", False, True), "bvugt": ("u", True, True), "bvule": ("u", False, False),
          "bvuge": ("u", True, False), "bvslt": ("s", False, True), "bvsgt": ("s", True, True),
          "bvsle": ("s", False, False), "bvsge": ("s", True, False)}


_M64 = (1 << 64) - 1


def _shash_args(ctx: Ctx, args) -> int:
    """A 64-bit structural hash of terms (op, width, params, value, name and
    the operands' hashes; stable across processes and contexts), memoised per
    node in the context."""
    memo = ctx.__dict__.setdefault("_shash", {})
    h = 0xCBF29CE484222325
    for a in args:
        h = ((h ^ _shash(a, memo)) * 0x100000001B3) & _M64
    return h


def _shash(root: Node, memo: Dict[int, int]) -> int:
    got = memo.get(root.id)
    if got is not None:
        return got
    for n in _unhashed(root, memo):
        h = zlib.crc32(n.op.encode())
        for x in (n.width, n.dom or 0, *n.params):
            h = ((h ^ (x & _M64)) * 0x100000001B3) & _M64
        if n.val is not None:
            v = n.val
            while True:
                h = ((h ^ (v & _M64)) * 0x100000001B3) & _M64
                v >>= 64
                if not v:
                    break
        if n.name is not None:
            h = ((h ^ zlib.crc32(n.name.encode())) * 0x100000001B3) & _M64
        for a in n.args:
            h = ((h ^ memo[a.id]) * 0x100000001B3 + 1) & _M64
        memo[n.id] = h
    return memo[root.id]


def _unhashed(root: Node, memo: Dict[int, int]) -> List[Node]:
    """the nodes under root with no hash yet, operands first"""
    out, stack = [], [(root, False)]
    seen = set()
    while stack:
        n, done = stack.pop()
        if done:
            out.append(n)
            continue
        if n.id in memo or n.id in seen:
            continue
        seen.add(n.id)
        stack.append((n, True))
        for a in reversed(n.args):
            if a.id not in memo and a.id not in seen:
                stack.append((a, False))
    return out


def _zeros(c: Ctx, n: int) -> List[Node]:
    return [c.const(0, min(MAXW, n - lo)) for lo in range(0, n, MAXW)]


def _offset(n: Node):
    """(base, k) with n == base + k (mod 2^w), for a const k, through nested
    constant additions (calldata offset + 4 + k: one base for every byte of
    the word); (n, 0) otherwise."""
    k = 0
    while n.op == "bvadd" and len(n.args) == 2:
        a, b = n.args
        if b.op == "const" and a.op != "const":
            n, k = a, k + b.val
        elif a.op == "const" and b.op != "const":
            n, k = b, k + a.val
        else:
            break
    return n, k & ((1 << n.width) - 1)


KEY_BIAS = 1 << 16      # _index_key: K - k + KEY_BIAS >= 0 for offsets k < 2^16
KEY_LIMIT = isa.IMPEQK_LIMIT   # premise constants the fused check carries (CHECK_IMPEQK)
KEY_MIN = 8             # premises a base needs before it is keyed (a key costs four instructions)
PAIR_TILE = 32   # symbolic cells kept resident while the concrete cells stream past


def _pair_order(reads):
    """Every unordered pair of one array's/function's reads, ordered for the
    register file: symbolic-symbolic pairs first, then the concrete x symbolic
    pairs in tiles of PAIR_TILE symbolic reads.  Within a tile each concrete
    cell is used PAIR_TILE times in a row and the tile's symbolic cells stay
    in registers, instead of the narrow file refilling one of 32+ live cells at
    every pair (C3: 2 371 -> ~300 fills).  With keyed premises (no premise
    flags live across the grid, _Rewriter.keyed) one tile holds an ABI word's
    32 bytes and each concrete cell dies after its 32 pairs (C3: 41 fills, one
    per spilled word; tile 12: 80; LASER corpus 153.5 k -> 152.8 k
    instructions)."""
    sym = [r for r in reads if not all(a.op == "const" for a in r.args)]
    con = [r for r in reads if all(a.op == "const" for a in r.args)]
    out = [(sym[i], sym[j]) for i in range(len(sym)) for j in range(i + 1, len(sym))]
    for k in range(0, len(sym), PAIR_TILE):
        tile = sym[k:k + PAIR_TILE]
        out += [(c, s) for c in con for s in tile]
    return out


def _pins(conjuncts: List[Node], ack: Dict[str, AckLeaf]) -> Dict[str, Node]:
    """{read name: K} for the top-level conjuncts (read = K) over a read's
    value leaf (Mythril's Power(256, k) = 256^k, keccak values of constant
    preimages): the congruence compares K instead of keeping the leaf live
    from that conjunct to the pair grid at the end of the program."""
    pins: Dict[str, Node] = {}
    for cj in _flatten(conjuncts):
        if cj.op != "=" or len(cj.args) != 2:
            continue
        x, k = cj.args
        if x.op == "const":
            x, k = k, x
        if k.op == "const" and x.op == "var" and x.name in ack and x.name not in pins:
            pins[x.name] = k
    return pins


def _narrow_imp(n: Node) -> bool:
    """n = (p => (x = y)) over narrow x, y: the shape CHECK_IMPEQK takes (a
    keyed premise before a wide compare would stay a flag, and its premise
    constant one of the asm interpreter's few narrow constant registers)"""
    if n.op != "=>":
        return False
    q = n.args[1]
    return q.op == "=" and len(q.args) == 2 and q.args[0].width <= 32


def _wide_index_eq(e: Node):
    """(base, K) for e = (base = K) with a symbolic base of 33..MAXW bits, else None"""
    if e.op != "=" or len(e.args) != 2:
        return None
    b, k = e.args
    if b.op == "const":
        b, k = k, b
    if k.op != "const" or b.op == "const" or not 32 < b.width <= MAXW:
        return None
    return b, k.val


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


def _topo_memo(roots: List[Node], seen: set, memo: dict, table: List[Node], whole: bool = False) -> List[Node]:
    """topo(roots, seen) from walks kept in ``memo`` (a long-lived context's):
    each root's own walk (whole=False: the main conjuncts, which share few
    nodes), or the fresh walk of the whole root list, keyed by its root ids
    (whole=True: the congruence conjuncts, thousands of small roots over the
    same few shared reads, identical while a set's reads are).  The same
    list as topo: a node ``seen`` before has its whole operand tree seen, so
    dropping the seen nodes from a fresh walk leaves exactly what the walk
    with ``seen`` emits, and a root's walk after earlier roots is its own
    walk without the nodes they emitted.  The merge is C-level
    (dict.fromkeys over ids; table is the context's node list, by id)."""
    if whole:
        key = tuple([r.id for r in roots])
        ids = memo.get(key)
        if ids is None:
            if len(memo) > _TOPO_MEMO_MAX:
                memo.clear()
            ids = memo[key] = tuple([n.id for n in topo(roots)])
    else:
        get = memo.get
        lists = []
        for r in roots:
            t = get(r.id)
            if t is None:
                t = memo[r.id] = tuple([n.id for n in topo([r])])
            lists.append(t)
        ids = dict.fromkeys(chain.from_iterable(lists))
    out = [i for i in ids if i not in seen] if seen else list(ids)
    seen.update(out)
    return list(map(table.__getitem__, out))


_TOPO_MEMO_MAX = 1 << 14
_ID = attrgetter("id")


def lower_constraints(conjuncts: List[Node], ctx: Ctx) -> Lowered:
    """Rewrite every conjunct, Ackermannise, add the congruence conjuncts.

    In a context marked ``long_lived`` (z3bridge.ConjunctCache's: one per
    Mythril process, where successor sets share their conjuncts) each
    conjunct's rewrite and the array / function reads it makes are kept
    (``ctx._lowered``, by conjunct id) and reused by every later set that
    holds it; only the congruence over the set's reads is built per query.
    Leaf names depend on the read alone (``_key_name``), so a rewrite is the
    same in every set, and the reads are collected in the order one walk of
    the whole set meets them: the program is the same either way."""
    lowered = ctx.__dict__.get("_lowered") if getattr(ctx, "long_lived", False) else None
    if lowered is None:
        rw = _Rewriter(ctx)
        out = [rw.rw(cj) for cj in conjuncts]
    else:
        out, ack = [], {}
        for cj in conjuncts:
            e = lowered.get(cj.id)
            if e is None:
                r1 = _Rewriter(ctx)
                e = lowered[cj.id] = (r1.rw(cj), list(r1.ack.values()))
            out.append(e[0])
            for al in e[1]:
                if al.name not in ack:
                    ack[al.name] = al
        rw = _Rewriter(ctx)
        rw.ack = ack
        for al in ack.values():
            rw.by_base.setdefault((al.kind, al.base), []).append(al)
    rw.pins = _pins(out, rw.ack)
    lists = None
    if lowered is not None:
        # the congruence and its keyed form depend on the reads per base (in
        # order) and the pinned values alone: kept per such key (a successor
        # that adds no read reuses its parent's lists outright)
        cmemo = ctx.__dict__.setdefault("_cong_lists", {})
        ckey = (tuple([(kb, tuple([al.name for al in reads])) for kb, reads in rw.by_base.items()]),
                tuple(sorted([(nm, k.id) for nm, k in rw.pins.items()])))
        lists = cmemo.get(ckey)
    if lists is None:
        cong = rw.congruence(ctx.__dict__.setdefault("_pairs", {}) if lowered is not None else None)
    else:
        cong = lists[0]
    fmain = _flatten(out)
    seen: set = set()
    if lowered is not None:        # per-root walks kept with the context (_topo_memo)
        tmemo = ctx.__dict__.setdefault("_topo", {})
        lmemo = ctx.__dict__.setdefault("_topo_lists", {})

        def walk(roots, seen_):
            return _topo_memo(roots, seen_, lmemo, ctx.nodes, whole=True)
        nmain = _topo_memo(fmain, seen, tmemo, ctx.nodes)
    else:
        walk = topo
        nmain = topo(fmain, seen)
    if lists is None:
        keyed = rw.keyed(cong, ctx.__dict__.setdefault("_keyed", {}) if lowered is not None else None)
    else:
        keyed = lists[1]
    seen_main = set(seen) if keyed is not cong else None
    fcong = _flatten(cong) if lists is None else lists[2]
    ncong = walk(fcong, seen)
    flat, nodes = fmain + fcong, nmain + ncong   # = topo(_flatten(out + cong))
    split = (len(nmain), tuple(map(_ID, ncong))) if lowered is not None and len(ncong) >= 256 else None
    if nodes and max(map(_width, nodes)) > MAXW:   # every consumer chunks its wide operands; none may remain
        n = next(n for n in nodes if n.width > MAXW)
        raise Unsupported(f"{n.width}-bit {n.op} outside the legalised vocabulary")
    fkeyed = None
    if keyed is not cong:
        fkeyed = _flatten(keyed) if lists is None else lists[3]
    if lists is None and lowered is not None:
        if len(cmemo) >= _TOPO_MEMO_MAX:
            cmemo.clear()
        cmemo[ckey] = (cong, keyed, fcong, fkeyed)
    if keyed is cong:
        return Lowered(out + cong, rw.ack, len(cong), flat, nodes, harvest_split=split)
    return Lowered(out + keyed, rw.ack, len(cong), fmain + fkeyed, nmain + walk(fkeyed, seen_main),
                   harvest_conjuncts=out + cong, harvest_nodes=nodes, harvest_split=split)


def needs_lowering(conjuncts: List[Node]) -> bool:
    for n in topo(conjuncts):
        if n.op in ("select", "apply", "store", "const_array", "array") or n.width > MAXW:
            return True
        if n.op in _POW2_OPS and len(n.args) == 2 and any(a.op == "const" for a in n.args):
            return True
    return False
