"""Candidate pools: which values each free variable is drawn from.

Random 256-bit draws almost never satisfy ``x == C`` (SURVEY.md §7 "hard parts"
4), so every leaf gets a pool of *interesting* values harvested from the
formula, mixed with RANDOM entries (Philox draws):

* values implied by comparisons against constants, projected through
  ``concat`` / ``extract`` / ``zero_extend`` / ``+K`` / ``-K`` / ``^K`` / ``ite``
  / ``udiv K`` / ``urem K`` down to the leaves (e.g. ``extract(255,224,
  concat(cd[0..31])) == 0xa9059cbb`` proposes ``cd[0]=0xa9 .. cd[3]=0xbb``),
  plus the constant +-1 for orderings;
* packed-array indexing: a term compared through both ``t / K == c`` and
  ``t % K == r`` (Solidity's packed ``bool[]``/``uint8[]`` reads: slot
  ``i / 32``, byte ``i % 32``, the byte offset reaching ``EXP`` / the ``Power``
  UF of ``exponent_function_manager.py``) gets the combined values ``c*K + r``
  first;
* the three LASER actors for 256-bit address-like leaves
  (``mythril/laser/ethereum/transaction/symbolic.py:29-40``: CREATOR
  0xAFFE.., ATTACKER 0xDEADBEEF.., SOMEGUY 0xAAAA..; the
  ``caller in ACTORS`` constraint of ``:210-212``);
* generic boundary values 0, 1, 2, 2^(w-1), 2^w-1 and width-truncated DAG
  constants.

Domain restriction (``domains``): facts that every model must satisfy are read
off the top-level conjuncts and shrink a leaf's pool to values that can
satisfy them, with no RANDOM entries:

* ``t == K`` where ``t`` projects injectively onto a leaf (concat / extract /
  zero_extend / ite with a differing constant arm / +K / ^K) fixes the leaf
  (the four selector bytes of a dispatcher JUMPI);
* ``t == K1 or t == K2 or ...`` fixing the same leaf in every disjunct gives
  that leaf the exact domain {K1, K2, ...} (``caller in ACTORS``,
  ``transaction/symbolic.py:210-212``);
* unsigned bounds ``K <= x``, ``x < K`` (and their negations) give an interval,
  and ``x mod K == 0`` an alignment; the pool becomes aligned values spread
  over the interval (``calldatasize`` bounds, the keccak UF intervals of
  ``keccak_function_manager.py:155-163``).

A disjunct that is the constant ``false`` is dropped first (``Or(cond, False)``
is how ``_create_condition`` reads with no concrete hashes).  Facts on a bare
leaf hold in every model; the ones read through an ``ite`` arm are heuristic.
Either way a pool only decides which candidates are tried: every witness is
re-checked, and a miss goes to z3.

Word ties (``_tie_words``): the byte leaves of one calldata word share one
word-level pool digit, so whole proposed words (an ABI offset, a count, 2^255)
are tried rather than byte mixtures.

Pools are laid out as index bit-fields while the 40 field bits last
(exhaustive enumeration of small spaces) and as hashed digits afterwards.
"""
from __future__ import annotations

import itertools
from typing import Dict, List, Optional, Tuple

from .compiler import LeafSpec
from .ir import BOOL, Node, topo

ACTORS = [0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE,
          0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF,
          0xAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAA]

_CMP = frozenset(("=", "distinct", "bvult", "bvule", "bvugt", "bvuge", "bvslt", "bvsle", "bvsgt", "bvsge"))
_ADDRESS_WORDS = ("sender", "caller", "origin", "creator", "address")


def _project(e: Node, value: int, out: Dict[str, List[int]], depth: int = 0,
             words: Optional[Dict[int, List[int]]] = None):
    """Propose leaf values that would make term e equal `value` (and, in
    `words`, whole values for every concat on the way)."""
    if depth > 24:
        return
    w = e.width
    if w == BOOL:
        return
    value &= (1 << w) - 1
    op = e.op
    if op == "var":
        out.setdefault(e.name, []).append(value)
    elif op == "concat":
        if words is not None:
            words.setdefault(e.id, []).append(value)
        off = w
        for a in e.args:
            off -= a.width
            _project(a, value >> off, out, depth + 1, words)
    elif op == "extract":
        hi, lo = e.params
        _project(e.args[0], value << lo, out, depth + 1, words)
    elif op in ("zero_extend", "sign_extend"):
        _project(e.args[0], value, out, depth + 1, words)
    elif op in ("bvadd", "bvsub", "bvxor") and len(e.args) == 2:
        a, b = e.args
        for x, k, xfirst in ((a, b, True), (b, a, False)):
            if k.op == "const":
                if op == "bvadd":
                    _project(x, value - k.val, out, depth + 1, words)
                elif op == "bvxor":
                    _project(x, value ^ k.val, out, depth + 1, words)
                elif xfirst:  # x - K = v  ->  x = v + K
                    _project(x, value + k.val, out, depth + 1, words)
                else:  # K - x = v -> x = K - v
                    _project(x, k.val - value, out, depth + 1, words)
    elif op == "ite":
        _project(e.args[1], value, out, depth + 1, words)
        _project(e.args[2], value, out, depth + 1, words)
    elif op in ("bvudiv", "bvurem") and e.args[1].op == "const" and e.args[1].val > 1:
        # x / K == v: the interval's start v*K; x % K == v: v itself
        _project(e.args[0], value * e.args[1].val if op == "bvudiv" else value, out, depth + 1, words)
    elif op in ("bvor", "bvand") and len(e.args) == 2:
        # a masked merge (an address written over a storage word's other bits):
        # either side may carry the value's bits
        for x in e.args:
            if x.op != "const":
                _project(x, value, out, depth + 1, words)


def _bare_leaf(t: Node) -> Optional[Node]:
    """The leaf under zero padding, low-bit extracts and constant masks, else None."""
    for _ in range(6):
        if t.op == "var":
            return t
        if t.op == "concat" and len(t.args) == 2 and t.args[0].op == "const" and t.args[0].val == 0:
            t = t.args[1]
        elif t.op == "zero_extend" or (t.op == "extract" and t.params[1] == 0):
            t = t.args[0]
        elif t.op == "bvand" and len(t.args) == 2 and (t.args[0].op == "const") != (t.args[1].op == "const"):
            t = t.args[1] if t.args[0].op == "const" else t.args[0]
        else:
            return None
    return None


def _assign(e: Node, value: int, lo: int, hi: int, out: Dict[str, List[int]], depth: int = 0) -> None:
    """Bits lo..hi of term e equal those bits of `value`: record, per leaf, the
    mask of bits this fixes and their values (partial fixes too, unlike
    ``_force``)."""
    if depth > 32 or e.width == BOOL or lo > hi:
        return
    op = e.op
    if op == "var":
        m = ((1 << (hi + 1)) - 1) ^ ((1 << lo) - 1)
        rec = out.setdefault(e.name, [0, 0, e.width])
        rec[0] |= m
        rec[1] = (rec[1] & ~m) | (value & m)
    elif op == "concat":
        off = e.width
        for a in e.args:
            off -= a.width
            a_lo, a_hi = max(lo, off), min(hi, off + a.width - 1)
            if a_lo <= a_hi:
                _assign(a, value >> off, a_lo - off, a_hi - off, out, depth + 1)
    elif op == "extract":
        _, l = e.params
        _assign(e.args[0], value << l, lo + l, hi + l, out, depth + 1)
    elif op == "zero_extend":
        x = e.args[0]
        _assign(x, value, lo, min(hi, x.width - 1), out, depth + 1)
    elif op == "ite":
        _, x, y = e.args
        for v, k in ((x, y), (y, x)):
            if k.op == "const" and v.op != "const":
                _assign(v, value, lo, hi, out, depth + 1)
                return
    elif op in ("bvudiv", "bvurem") and e.args[1].op == "const" and e.args[1].val > 1 and lo == 0 \
            and hi == e.width - 1 and e.args[1].val & (e.args[1].val - 1) == 0:
        k = e.args[1].val.bit_length() - 1       # powers of two: a bit field of the dividend
        x = e.args[0]
        if op == "bvudiv":
            _assign(x, value << k, k, x.width - 1, out, depth + 1)
        else:
            _assign(x, value, 0, k - 1, out, depth + 1)


def _combine_partial(facts: List[Dict[str, List[int]]]) -> List[Dict[str, int]]:
    """Packed-array indexing (module doc): pairs of facts that each fix only
    some bits of a shared leaf, fix disjoint bits of it and agree elsewhere,
    merged into one assignment of full leaf values (unfixed bits 0)."""
    partial = facts
    by_leaf: Dict[str, List[int]] = {}
    for i, f in enumerate(partial):
        for name in f:
            by_leaf.setdefault(name, []).append(i)
    out, seen = [], set()
    for name, idx in by_leaf.items():
        idx = idx[:96]
        for ii, i in enumerate(idx):
            for j in idx[ii + 1:]:
                if (i, j) in seen:
                    continue
                seen.add((i, j))
                a, b = partial[i], partial[j]
                if a[name][0] & b[name][0] or a[name][0] | b[name][0] == a[name][0] or \
                        a[name][0] | b[name][0] == b[name][0]:
                    continue          # the same bits of the shared leaf: not complementary
                ok = all((a[n][0] & b[n][0] & (a[n][1] ^ b[n][1])) == 0 for n in a if n in b)
                if ok:
                    merged = {n: a.get(n, [0, 0])[1] | b.get(n, [0, 0])[1] for n in set(a) | set(b)}
                    out.append(merged)
                if len(out) >= 256:
                    return out
    return out


def _force(e: Node, value: int, lo: int, hi: int, out: Dict[str, int], depth: int = 0) -> None:
    """Bits lo..hi of term e must equal those bits of `value`; record every leaf
    whose bits are all fixed that way."""
    if depth > 32 or e.width == BOOL or lo > hi:
        return
    w = e.width
    op = e.op
    if op == "var":
        if lo == 0 and hi == w - 1:
            out.setdefault(e.name, value & ((1 << w) - 1))
    elif op == "concat":
        off = w
        for a in e.args:
            off -= a.width
            a_lo, a_hi = max(lo, off), min(hi, off + a.width - 1)
            if a_lo <= a_hi:
                _force(a, value >> off, a_lo - off, a_hi - off, out, depth + 1)
    elif op == "extract":
        _, l = e.params
        _force(e.args[0], value << l, lo + l, hi + l, out, depth + 1)
    elif op == "zero_extend":
        x = e.args[0]
        _force(x, value, lo, min(hi, x.width - 1), out, depth + 1)
    elif op == "ite":
        rng = ((1 << (hi + 1)) - 1) ^ ((1 << lo) - 1)
        _, a, b = e.args
        if b.op == "const" and (b.val ^ value) & rng:
            _force(a, value, lo, hi, out, depth + 1)
        elif a.op == "const" and (a.val ^ value) & rng:
            _force(b, value, lo, hi, out, depth + 1)
    elif op in ("bvadd", "bvxor") and len(e.args) == 2 and lo == 0 and hi == w - 1:
        a, b = e.args
        for x, k in ((a, b), (b, a)):
            if k.op == "const" and x.op != "const":
                _force(x, value - k.val if op == "bvadd" else value ^ k.val, lo, hi, out, depth + 1)


def _align_of(t: Node):
    """(leaf name, K) when ``t == 0`` says the leaf is a multiple of K: the
    ``bvurem(x, K)`` form and its power-of-two rewrite ``concat(0, extract(j-1, 0, x))``
    (lower.py, z3 simplify's shape), or a bare low-bit extract."""
    if t.op == "bvurem" and t.args[0].op == "var" and t.args[1].op == "const" and t.args[1].val > 1:
        return t.args[0].name, t.args[1].val
    if t.op == "concat" and len(t.args) == 2 and t.args[0].op == "const" and t.args[0].val == 0:
        t = t.args[1]
    if t.op == "extract" and t.params[1] == 0 and t.args[0].op == "var" and t.params[0] + 1 < t.args[0].width:
        return t.args[0].name, 1 << (t.params[0] + 1)
    return None


def _eq_const(n: Node):
    if n.op == "=" and len(n.args) == 2:
        a, b = n.args
        if b.op == "const" and a.op != "const":
            return a, b.val
        if a.op == "const" and b.op != "const":
            return b, a.val
    return None


_UPPER = {"bvult": (0, -1), "bvule": (0, 0), "bvugt": (1, -1), "bvuge": (1, 0)}


def domains(conjuncts: List[Node]):
    """Exact domains, unsigned intervals and alignments implied by the top-level
    conjuncts (module doc).  Returns (exact: name -> [values], interval: name ->
    [lo, hi] inclusive, align: name -> K)."""
    exact: Dict[str, List[int]] = {}
    interval: Dict[str, List[int]] = {}
    align: Dict[str, int] = {}
    below: List[tuple] = []          # (x, y, strict): leaf x <=u / <u leaf y

    def facts(n: Node, neg: bool = False):
        if n.op == "not":
            facts(n.args[0], not neg)
            return
        if n.op == ("or" if neg else "and"):
            for a in n.args:
                facts(a, neg)
            return
        if n.op == ("and" if neg else "or"):
            live = [a for a in n.args if not (a.op == "const" and bool(a.val) == neg)]
            if len(live) == 1:
                facts(live[0], neg)
                return
            if neg:
                return
            per = []
            for a in live:
                ec = _eq_const(a)
                f: Dict[str, int] = {}
                if ec is not None:
                    _force(ec[0], ec[1], 0, ec[0].width - 1, f)
                per.append(f)
            if per:
                for name in set(per[0]).intersection(*per[1:]):
                    vals = list(dict.fromkeys(f[name] for f in per))
                    if name not in exact or len(vals) < len(exact[name]):
                        exact[name] = vals
            return
        if neg:
            if n.op in _UPPER:   # not (a < b) == (b <= a), etc.
                a, b = n.args
                flip = {"bvult": "bvule", "bvule": "bvult", "bvugt": "bvuge", "bvuge": "bvugt"}[n.op]
                _bound(flip, b, a)
            return
        ec = _eq_const(n)
        if ec is not None:
            f: Dict[str, int] = {}
            _force(ec[0], ec[1], 0, ec[0].width - 1, f)
            for name, v in f.items():
                exact[name] = [v]
            t, k = ec
            al = _align_of(t) if k == 0 else None
            if al is not None:
                align[al[0]] = al[1]
            return
        if n.op in _UPPER:
            _bound(n.op, *n.args)

    def _shifted(t: Node):
        """(leaf, d) when t is leaf + d (bvadd/bvsub with a constant), else None."""
        if t.op == "var":
            return t, 0
        if t.op in ("bvadd", "bvsub") and len(t.args) == 2:
            x, k = t.args
            if x.op == "var" and k.op == "const":
                return x, (k.val if t.op == "bvadd" else -k.val)
            if t.op == "bvadd" and k.op == "var" and x.op == "const":
                return k, x.val
        return None

    def _bound(op, a, b):
        # op(a, b) holds; normalise to x (+ d) <= K or K <= x (+ d).  Offsets move
        # the bound without modelling wrap-around: the interval only steers the
        # pools (every candidate is still checked exactly)
        upper, strict = _UPPER[op]   # bvult/bvule: a is below b
        lo_t, hi_t = (b, a) if upper else (a, b)
        xl, xh = _bare_leaf(lo_t), _bare_leaf(hi_t)
        if xl is not None and xh is not None and xl is not xh:
            below.append((xl.name, xh.name, strict == -1))   # lo_t is the smaller side
        sl, sh = _shifted(lo_t), _shifted(hi_t)
        if sl is not None and hi_t.op == "const":       # x + d <(=) K
            x, d = sl
            top = hi_t.val + strict - d
            if 0 <= top < (1 << x.width):
                iv = interval.setdefault(x.name, [0, (1 << x.width) - 1])
                iv[1] = min(iv[1], top)
        elif sh is not None and lo_t.op == "const":     # K <(=) x + d
            x, d = sh
            bot = lo_t.val - strict - d
            if 0 <= bot < (1 << x.width):
                iv = interval.setdefault(x.name, [0, (1 << x.width) - 1])
                iv[0] = max(iv[0], bot)

    for c in conjuncts:
        facts(c)
    domains.below = below
    return exact, interval, align


def _pad_pow2(vals: List[int]) -> List[int]:
    n = 1
    while n < len(vals):
        n *= 2
    return [vals[i % len(vals)] for i in range(n)]


def _restrict(pool: List[Optional[int]], name: str, w: int, exact, interval, align, pool_size: int,
              props=()):
    lo, hi = interval.get(name, (0, (1 << w) - 1))
    K = align.get(name, 1)
    ok = lambda v: lo <= v <= hi and v % K == 0   # noqa: E731
    if name in exact:
        vals = [v for v in exact[name] if ok(v)]
        return _pad_pow2(vals) if vals else pool
    if name not in interval and name not in align:
        return pool
    first = lo + (-lo % K)
    if first > hi:
        return pool
    last = hi - (hi % K)
    keep = [v for v in pool if v is not None and ok(v)]
    steps = (last - first) // K
    spread = [first + (steps * i // 16) * K for i in range(1, 16)]
    # Pool order is search order, and with many leaves only the first two
    # entries vary below 2^24.  Bounds first, then the largest harvested
    # proposal below 2^(w-1), the signed maximum (above every signed guard,
    # where the upper bound 2^w-1 is -1), the bounds' neighbours, the other
    # harvested values and values spread over the interval.  A calldatasize
    # (calldata.py:214-231) leads with that proposal instead: the highest guard
    # `i <s size` of a calldata read, so every argument byte reads (0x44 for two
    # ABI words); the lower bound (selector only) and 2^w-1 (nothing reads, not
    # even the selector) follow.
    # (a proposal at most one step above the lower bound is that bound's own +-1)
    pos = [v for v in props if ok(v) and first + K < v < (1 << (w - 1)) and v != last] if w >= 2 else []
    top = [max(pos)] if pos else []
    smax = [(1 << (w - 1)) - 1] if w >= 2 else []
    head = top + [first, last] if name.endswith("calldatasize") else [first, last] + top
    vals = list(dict.fromkeys(v for v in head + smax + [first + K, last - K] + keep[:8]
                              + spread + keep[8:] if ok(v)))[:pool_size]
    if steps + 1 > len(vals) and (hi - lo) >= (1 << max(w - 2, 0)) and K == 1:
        return vals + [None] * max(1, pool_size // 4)   # wide interval: random draws still land often
    return _pad_pow2(vals)   # no RANDOM padding: a random draw would almost never satisfy the facts


def _const_props(consts, m: int, split_bytes: bool):
    for c in consts:
        yield c & m
        if split_bytes:
            for i in range(min(32, (c.bit_length() + 7) // 8)):
                yield (c >> (8 * i)) & 0xFF


def _cmp_effect(n: Node):
    """What one comparison node contributes to harvest: the proposals its
    constant side projects onto leaves (per leaf, in order), the whole-word
    proposals of the concats on the way, and (for =) the partial bit fixes."""
    op = n.op
    props: Dict[str, List[int]] = {}
    words: Dict[int, List[int]] = {}
    part: List[Dict[str, List[int]]] = []
    a, b = n.args
    for x, k in ((a, b), (b, a)):
        if k.op == "const" and x.op != "const":
            deltas = (0,) if op in ("=", "distinct") else (0, 1, -1)
            for d in deltas:
                _project(x, k.val + d, props, words=words)
            if op == "=" and x.width != BOOL:
                f: Dict[str, List[int]] = {}
                _assign(x, k.val, 0, x.width - 1, f)
                if any(m != (1 << w) - 1 for m, _, w in f.values()):
                    part.append(f)
    return props, words, part


_SEG_MEMO_MAX = 64


def _scan(nodes: List[Node], memo: Optional[dict]):
    """harvest's walk over one segment of the node list, as lists in node
    order: constants, vars, concats, the comparisons' contributions
    (_cmp_effect, non-empty ones), alignment facts (leaf, K) and leaf
    unions (name, name).  The unions of a segment are reduced to one edge
    per merged name (same partition: harvest's proposals depend on the
    partition alone, not on its union order)."""
    consts, vars_, concats, effs, align, unions = [], [], [], [], [], []
    for n in nodes:
        op = n.op
        if op == "const":
            if n.width != BOOL:
                consts.append(n.val)
            continue
        if op == "var":
            vars_.append(n)
            continue
        if op == "concat":
            concats.append(n)
            continue
        if op in _CMP and len(n.args) == 2:
            eff = memo.get(n.id) if memo is not None else None
            if eff is None:
                eff = _cmp_effect(n)
                if memo is not None:
                    memo[n.id] = eff
            if eff[0] or eff[1] or eff[2]:
                effs.append(eff)
            if op == "=":
                a, b = n.args
                for x, k in ((a, b), (b, a)):
                    al = _align_of(x) if (k.op == "const" and k.val == 0) else None
                    if al is not None:
                        align.append(al)
                # x = y, also through the masks and zero-padding of an address
                # compare (concat(0, extract(159, 0, x)), bvand(mask, x)): a stored
                # owner equated with msg.sender gets the actors
                xa, xb = _bare_leaf(a), _bare_leaf(b)
                if xa is not None and xb is not None and xa.width == xb.width and xa is not xb:
                    unions.append((xa.name, xb.name))
    if len(unions) > 8:
        parent: Dict[str, str] = {}

        def find(x):
            while parent.get(x, x) != x:
                parent[x] = parent.get(parent[x], parent[x])
                x = parent[x]
            return x
        for na, nb in unions:
            ra, rb = find(na), find(nb)
            if ra != rb:
                parent[ra] = rb
        unions = [(x, find(x)) for x in parent]
    return consts, vars_, concats, effs, align, unions


def harvest(conjuncts: List[Node], leaves: Optional[List[Node]], pool_size: int = 32,
            random_share: float = 0.25, restrict: bool = True,
            nodes: Optional[List[Node]] = None, memo: Optional[dict] = None,
            split: Optional[Tuple[int, tuple]] = None) -> Dict[str, LeafSpec]:
    """nodes: topo(conjuncts) when the caller has it (prepare: Lowered.nodes,
    the same walk without the top-level `and` nodes, which no rule reads).
    leaves None: every var of `nodes`, first occurrence of each name in walk
    order (collected by the same loop that reads the constants).
    memo: a dict kept with a long-lived context (engine.prepare passes the
    context's), holding each comparison node's contribution (_cmp_effect):
    the same proposals in the same order, computed once per node."""
    if nodes is None:
        nodes = topo(conjuncts)
    collect = leaves is None
    if collect:
        leaves = []
        seen_leaf = set()
    exact, interval, dom_align = domains(conjuncts) if restrict else ({}, {}, {})
    proposals: Dict[str, List[int]] = {}
    # orderings between two leaves (INVEST_MIN < msg.value < INVEST_MAX with
    # symbolic storage): each leaf leads with its rank in the order, so the
    # first candidates already respect it (0 < 1 < 2 ...)
    ranks: Dict[str, int] = {}
    below = getattr(domains, "below", []) if restrict else []
    for _ in range(8):
        changed = False
        for small, big, strict in below:
            r = ranks.get(small, 0) + (1 if strict else 0)
            if ranks.get(big, 0) < r:
                ranks[big] = r
                changed = True
            ranks.setdefault(small, 0)
        if not changed:
            break
    for name, r in ranks.items():
        proposals[name] = [r]
    word_props: Dict[int, List[int]] = {}
    consts = []
    dm: List[Dict[str, List[int]]] = []
    concats: List[Node] = []  # word candidates (_tie_words)
    align: Dict[str, int] = {}
    unions: List[Tuple[str, str]] = []
    # the node list in segments: (start, end, memo key or None).  A keyed
    # segment's scan (_scan) is kept in the context's memo and replayed: the
    # accumulators below only ever append in node order, so replaying a
    # segment's lists equals scanning its nodes again (split: engine.prepare
    # passes Lowered.harvest_split, the congruence part of a long-lived set)
    if split is not None and memo is not None:
        segs = [(0, split[0], None), (split[0], len(nodes), ("seg", split[1]))]
    else:
        segs = [(0, len(nodes), None)]
    for a, b, key in segs:
        sc = memo.get(key) if key is not None else None
        if sc is None:
            sc = _scan(nodes[a:b] if (a, b) != (0, len(nodes)) else nodes, memo)
            if key is not None:
                segm = memo.setdefault("segments", [])
                if len(segm) >= _SEG_MEMO_MAX:      # bounded: a long run meets many read sets
                    memo.pop(segm.pop(0), None)
                segm.append(key)
                memo[key] = sc
        s_consts, s_vars, s_concats, s_effs, s_align, s_unions = sc
        consts.extend(s_consts)
        if collect:
            for n in s_vars:
                if n.name not in seen_leaf:
                    seen_leaf.add(n.name)
                    leaves.append(n)
        concats.extend(s_concats)
        for props, words, part in s_effs:
            for name, vs in props.items():
                got = proposals.get(name)
                if got is None:
                    proposals[name] = list(vs)
                else:
                    got.extend(vs)
            for wid, vs in words.items():
                got = word_props.get(wid)
                if got is None:
                    word_props[wid] = list(vs)
                else:
                    got.extend(vs)
            dm.extend(part)                    # facts fixing only part of some leaf's bits
        for name, K in s_align:
            align[name] = K
        unions.extend(s_unions)
    # packed-array indexing: t / K == c and t % K == r -> t = c*K + r, tried first
    combos = _combine_partial(dm)
    # alignment facts: (= (bvurem x K) 0)  ->  x should be a multiple of K (_scan)
    for name, K in align.items():
        props = proposals.get(name, [])
        aligned = []
        for v in props:
            up = v + (-v % K)
            aligned += [up, up + K, up + 2 * K]
        proposals[name] = aligned + props
    # leaves equated with each other share their proposals (union-find over var = var)
    parent: Dict[str, str] = {}

    def find(x):
        while parent.get(x, x) != x:
            parent[x] = parent.get(parent[x], parent[x])
            x = parent[x]
        return x

    for na, nb in unions:     # x = y between two leaves (_scan)
        ra, rb = find(na), find(nb)
        if ra != rb:
            parent[ra] = rb
    if parent:
        groups: Dict[str, List[int]] = {}
        for name, props in list(proposals.items()):
            groups.setdefault(find(name), []).extend(props)
        members: Dict[str, int] = {}
        for name in set(parent) | set(proposals):
            r = find(name)
            members[r] = members.get(r, 0) + 1
        uniq: Dict[str, List[int]] = {}   # each group's proposals, first occurrences, once
        for name in list(parent) + list(proposals):
            r = find(name)
            # a group of one keeps its proposals as they are: the pool below
            # takes first occurrences anyway, and _restrict only their maximum
            merged = groups.get(r) if members[r] > 1 else None
            if merged:
                du = uniq.get(r)
                if du is None:
                    du = uniq[r] = list(dict.fromkeys(merged))
                # = dict.fromkeys(own + merged): own first, then the group's others
                own = dict.fromkeys(proposals.get(name, ()))
                proposals[name] = list(own) + [v for v in du if v not in own]
    specs: Dict[str, LeafSpec] = {}
    uniq_consts = list(dict.fromkeys(consts))[:256]
    tails: Dict[int, List[int]] = {}   # width -> the constants' proposals, deduplicated
    plain_pools: Dict[int, List[int]] = {}   # width -> the pool of a leaf with no proposals of its own
    nfixed = max(1, int(pool_size * (1 - random_share)))
    # word ties first: their bytes' pools are the word's (no pool of their own to build)
    tied = _tie_words(concats, {lf.name for lf in leaves if lf.op == "var"}, word_props, set(exact), uniq_consts,
                      pool_size, random_share, combos)
    for leaf in leaves:
        if leaf.op != "var":
            continue
        t = tied.get(leaf.name)
        if t is not None:
            specs[leaf.name] = t
            continue
        w = 1 if leaf.width == BOOL else leaf.width
        m = (1 << w) - 1
        actors = ACTORS if w >= 160 and any(t in leaf.name.lower() for t in _ADDRESS_WORDS) else ()
        # lazily: the pool fills after a few dozen values, and the byte split of
        # 256 constants for every calldata byte leaf was most of prepare()'s time
        props = proposals.get(leaf.name, ())
        plain = not props and not actors and not (combos and any(leaf.name in c for c in combos))
        got = plain_pools.get(w) if plain else None     # a leaf nothing proposes: its width's pool
        if got is not None:
            pool = list(got)
        else:
            tail = tails.get(w)
            if tail is None:
                tail = tails[w] = list(dict.fromkeys(_const_props(uniq_consts, m, w == 8)))
            cand = itertools.chain(props, actors, (0, 1, 2, m, 1 << (w - 1), m - 1), tail)
            pool = []
            seen = set()
            add, put, k = seen.add, pool.append, 0
            for v in itertools.chain((c[leaf.name] for c in combos if leaf.name in c), cand) if combos else cand:
                v &= m
                if v not in seen:
                    add(v)
                    put(v)
                    k += 1
                    if k >= nfixed:
                        break
            if plain:
                plain_pools[w] = list(pool)
        if w == 1:
            pool = [0, 1]
        else:
            nrand = max(1, pool_size - len(pool)) if len(pool) >= nfixed else max(1, len(pool) // 3)
            pool += [None] * nrand
            if restrict:
                pool = _restrict(pool, leaf.name, w, exact, interval, dom_align, pool_size,
                                 proposals.get(leaf.name, ()))
        specs[leaf.name] = LeafSpec(leaf.name, w, pool=pool)
    return specs


# ABI head values: offsets of dynamic arguments are small multiples of 32
ABI_WORDS = [0x20, 0x40, 0x60, 0x80, 0xA0, 0xC0]


def _byte_leaf(a: Node) -> Optional[Node]:
    """The 8-bit leaf a concat argument reads: ``x`` or ``ite(g, x, K)`` (a
    calldata byte behind its ``index < calldatasize`` guard, calldata.py:218-231)."""
    if a.op == "var" and a.width == 8:
        return a
    if a.op == "ite":
        _, x, y = a.args
        for v, k in ((x, y), (y, x)):
            if v.op == "var" and v.width == 8 and k.op == "const":
                return v
    return None


def _tie_words(nodes, names, word_props, exact_names, uniq_consts, pool_size, random_share, combos=()):
    """Bytes of one word (a concat of byte leaves: an ABI argument read from
    calldata, ``calldata.py:218-231``) draw one word-level pool entry together:
    the pool holds whole-word proposals split into bytes, and every byte after
    the first copies the first's digit (LeafSpec.tie).  Without this each byte
    picks its own entry and a proposed word value (an array offset, a count) is
    hit with probability |pool|^-31.  Bytes already fixed by a domain fact stay
    singletons; a byte joins at most one word, the one with most free bytes.
    names: the leaves that get a spec; returns {byte leaf name: its spec}."""
    specs: Dict[str, LeafSpec] = {}
    words = []
    for n in nodes:
        if n.op == "concat" and len(n.args) >= 2:
            bl = [_byte_leaf(a) for a in n.args]
            if all(b is not None for b in bl) and len({b.name for b in bl}) == len(bl):
                words.append((n, bl))
    taken = set(exact_names)
    nfixed = max(1, int(pool_size * (1 - random_share)))
    while words:
        scored = []
        for n, bl in words:
            f = [(i, b) for i, b in enumerate(bl) if b.name not in taken and b.name in names]
            if len(f) >= 2:   # a word with fewer free bytes never regains them
                scored.append(((len(f), len(word_props.get(n.id, ()))), n, bl, f))
        if not scored:
            break
        best = max(scored, key=lambda x: x[0])
        _, n, bl, fb = best
        words = [(m, ml) for _, m, ml, _ in scored if m is not n]
        W = n.width
        m = (1 << W) - 1
        generic = {0, 1, 2, m, m - 1, 1 << (W - 1)}
        props = [v for v in dict.fromkeys(v & m for v in word_props.get(n.id, [])) if v not in generic]
        # merged partial facts (packed-array indexing) that reach this word come first
        nb_ = len(bl)
        lead_combos = []
        for cmb in combos:
            if any(b.name in cmb for _, b in fb):
                lead_combos.append(sum(cmb.get(b.name, 0) << (8 * (nb_ - 1 - i)) for i, b in enumerate(bl)))
        props = list(dict.fromkeys(lead_combos + props))
        abi = ABI_WORDS if any("calldata" in b.name for _, b in fb) else []
        # Pool order is search order (Morton digits try low entries first), so
        # the first few proposals, an ABI offset and the extreme values come
        # before the rest: a crowd of proposals (e.g. from congruence
        # side-conditions) must not push them out of the early indices.
        cand = props[:2] + abi[1:2] + [1 << (W - 1), m] + props[2:4] + [0, 1] + abi[2:] + abi[:1] \
            + [2, m - 1] + props[4:] + [c & m for c in uniq_consts]
        pool: List[Optional[int]] = list(dict.fromkeys(v & m for v in cand))[:nfixed]
        pool += [None] * max(1, pool_size - nfixed)
        nb = len(bl)
        lead = fb[0][1].name
        for i, b in fb:
            sh = 8 * (nb - 1 - i)
            specs[b.name] = LeafSpec(b.name, 8, pool=[None if v is None else (v >> sh) & 0xFF for v in pool],
                                     tie=None if b.name == lead else lead)
            taken.add(b.name)
    return specs
