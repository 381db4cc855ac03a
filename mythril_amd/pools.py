"""Candidate pools: which values each free variable is drawn from.

Random 256-bit draws almost never satisfy ``x == C`` (SURVEY.md §7 "hard parts"
4), so every leaf gets a pool of *interesting* values harvested from the
formula, mixed with RANDOM entries (Philox draws):

* values implied by comparisons against constants, projected through
  ``concat`` / ``extract`` / ``zero_extend`` / ``+K`` / ``-K`` / ``^K`` / ``ite``
  down to the leaves (e.g. ``extract(255,224, concat(cd[0..31])) == 0xa9059cbb``
  proposes ``cd[0]=0xa9 .. cd[3]=0xbb``), plus the constant +-1 for orderings;
* the three LASER actors for 256-bit address-like leaves
  (``mythril/laser/ethereum/transaction/symbolic.py:29-40``: CREATOR
  0xAFFE.., ATTACKER 0xDEADBEEF.., SOMEGUY 0xAAAA..; the
  ``caller in ACTORS`` constraint of ``:210-212``);
* generic boundary values 0, 1, 2, 2^(w-1), 2^w-1 and width-truncated DAG
  constants.

Pools are laid out as index bit-fields while the 40 field bits last
(exhaustive enumeration of small spaces) and as hashed digits afterwards.
"""
from __future__ import annotations

from typing import Dict, List, Optional

from .compiler import LeafSpec
from .ir import BOOL, Node, topo

ACTORS = [0xAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFEAFFE,
          0xDEADBEEFDEADBEEFDEADBEEFDEADBEEFDEADBEEF,
          0xAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAAA]

_CMP = ("=", "distinct", "bvult", "bvule", "bvugt", "bvuge", "bvslt", "bvsle", "bvsgt", "bvsge")


def _project(e: Node, value: int, out: Dict[str, List[int]], depth: int = 0):
    """Propose leaf values that would make term e equal `value`."""
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
        off = w
        for a in e.args:
            off -= a.width
            _project(a, value >> off, out, depth + 1)
    elif op == "extract":
        hi, lo = e.params
        _project(e.args[0], value << lo, out, depth + 1)
    elif op in ("zero_extend", "sign_extend"):
        _project(e.args[0], value, out, depth + 1)
    elif op in ("bvadd", "bvsub", "bvxor") and len(e.args) == 2:
        a, b = e.args
        for x, k, xfirst in ((a, b, True), (b, a, False)):
            if k.op == "const":
                if op == "bvadd":
                    _project(x, value - k.val, out, depth + 1)
                elif op == "bvxor":
                    _project(x, value ^ k.val, out, depth + 1)
                elif xfirst:  # x - K = v  ->  x = v + K
                    _project(x, value + k.val, out, depth + 1)
                else:  # K - x = v -> x = K - v
                    _project(x, k.val - value, out, depth + 1)
    elif op == "ite":
        _project(e.args[1], value, out, depth + 1)
        _project(e.args[2], value, out, depth + 1)


def harvest(conjuncts: List[Node], leaves: List[Node], pool_size: int = 32,
            random_share: float = 0.25) -> Dict[str, LeafSpec]:
    nodes = topo(conjuncts)
    proposals: Dict[str, List[int]] = {}
    consts = []
    for n in nodes:
        if n.op == "const" and n.width != BOOL:
            consts.append(n.val)
        if n.op in _CMP and len(n.args) == 2:
            a, b = n.args
            for x, k in ((a, b), (b, a)):
                if k.op == "const" and x.op != "const":
                    deltas = (0,) if n.op in ("=", "distinct") else (0, 1, -1)
                    for d in deltas:
                        _project(x, k.val + d, proposals)
    # alignment facts: (= (bvurem x K) 0)  ->  x should be a multiple of K
    align: Dict[str, int] = {}
    for n in nodes:
        if n.op == "=" and len(n.args) == 2:
            a, b = n.args
            for x, k in ((a, b), (b, a)):
                if k.op == "const" and k.val == 0 and x.op == "bvurem" and x.args[1].op == "const" \
                        and x.args[0].op == "var" and x.args[1].val > 1:
                    align[x.args[0].name] = x.args[1].val
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

    for n in nodes:
        if n.op == "=" and len(n.args) == 2 and all(a.op == "var" for a in n.args) \
                and n.args[0].width == n.args[1].width:
            ra, rb = find(n.args[0].name), find(n.args[1].name)
            if ra != rb:
                parent[ra] = rb
    groups: Dict[str, List[int]] = {}
    for name, props in list(proposals.items()):
        groups.setdefault(find(name), []).extend(props)
    for name in list(parent) + list(proposals):
        merged = groups.get(find(name))
        if merged:
            proposals[name] = list(dict.fromkeys(proposals.get(name, []) + merged))
    specs: Dict[str, LeafSpec] = {}
    uniq_consts = list(dict.fromkeys(consts))[:256]
    for leaf in leaves:
        if leaf.op != "var":
            continue
        w = 1 if leaf.width == BOOL else leaf.width
        m = (1 << w) - 1
        cand: List[int] = []
        cand += proposals.get(leaf.name, [])
        lname = leaf.name.lower()
        if w >= 160 and any(t in lname for t in ("sender", "caller", "origin", "creator", "address")):
            cand += ACTORS
        cand += [0, 1, 2, m, 1 << (w - 1), m - 1]
        for c in uniq_consts:
            cand.append(c & m)
            if w == 8:
                cand.extend((c >> (8 * i)) & 0xFF for i in range(min(32, (c.bit_length() + 7) // 8)))
        pool: List[Optional[int]] = []
        seen = set()
        nfixed = max(1, int(pool_size * (1 - random_share)))
        for v in cand:
            v &= m
            if v not in seen:
                seen.add(v)
                pool.append(v)
            if len(pool) >= nfixed:
                break
        if w == 1:
            pool = [0, 1]
        else:
            nrand = max(1, pool_size - len(pool)) if len(pool) >= nfixed else max(1, len(pool) // 3)
            pool += [None] * nrand
        specs[leaf.name] = LeafSpec(leaf.name, w, pool=pool)
    return specs
