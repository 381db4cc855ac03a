"""Synthetic constraint DAGs (BASELINE.json config C5).

C5: a 10 000-node 256-bit bitvector DAG over 16 free 256-bit variables whose
root is the AND of 32 comparisons, with a planted witness.  Op mix by weight
(SURVEY.md §8d): add 15, sub 10, mul 10, and/or/xor 15, shl/lshr/ashr 10,
ult/ule/slt/eq 15, ite 10, extract/concat/zero_extend 10, udiv/urem 5.
Candidate leaf values are Philox4x32-10 draws (random leaves).

Shape: 32 chains; every node takes the previous node of its chain as one
operand and, as the other, a recent node of the same chain, a leaf, or a
constant — so all 10k nodes are reachable from the root and the live set
stays small (as in Mythril path constraints, which are shallow trees over the
transaction leaves).  Comparison results feed the next ``ite`` of the chain.

Planting: chain i ends in ``bvult(c_i, T_i)`` with T_i chosen from c_i's
value at the witness index so that the witness satisfies every conjunct and
each conjunct holds for a fraction ~2^(-density_log2/32) of candidates.  The
chain values at the witness come from a caller-supplied ``evaluate`` (the GPU
engine in bench.py, the host emulator or oracle in tests).
"""
from __future__ import annotations

import random
from dataclasses import dataclass
from typing import Callable, List, Sequence

from .ir import BOOL, Ctx, Node

M256 = (1 << 256) - 1

C5_WEIGHTS = [
    ("bvadd", 15), ("bvsub", 10), ("bvmul", 10), ("logic", 15), ("shift", 10),
    ("cmp", 15), ("ite", 10), ("struct", 10), ("div", 5),
]


@dataclass
class Synthetic:
    ctx: Ctx
    leaves: List[Node]
    chain_ends: List[Node]
    conjuncts: List[Node]
    witness_index: int
    seed: int
    n_nodes: int


def _pick(r: random.Random, weights):
    tot = sum(w for _, w in weights)
    x = r.uniform(0, tot)
    for name, w in weights:
        x -= w
        if x <= 0:
            return name
    return weights[-1][0]


def build_chains(n_nodes: int = 10000, n_leaves: int = 16, n_conj: int = 32, seed: int = 0x5EED0005,
                 window: int = 6):
    r = random.Random(seed)
    ctx = Ctx()
    leaves = [ctx.var(f"x{i}", 256) for i in range(n_leaves)]
    per_chain = max(4, (n_nodes - 2 * n_conj) // n_conj)
    count = 0
    ends: List[Node] = []
    pend_bools: List[List[Node]] = []

    def mk(op, *args, params=()):
        nonlocal count
        count += 1
        return ctx.app(op, *args, params=params)

    for ci in range(n_conj):
        prev = r.choice(leaves)
        recent: List[Node] = [prev]
        bools: List[Node] = []
        start = count
        while count - start < per_chain:
            def other():
                x = r.random()
                if x < 0.45 and recent:
                    return r.choice(recent[-window:])
                if x < 0.85:
                    return r.choice(leaves)
                return ctx.const(r.getrandbits(256), 256)
            kind = _pick(r, C5_WEIGHTS)
            if kind in ("bvadd", "bvsub", "bvmul"):
                nxt = mk(kind, prev, other())
            elif kind == "logic":
                nxt = mk(r.choice(["bvand", "bvor", "bvxor"]), prev, other())
            elif kind == "shift":
                amt = r.random()
                sh = ctx.const(r.randrange(1, 256), 256) if amt < 0.5 else mk("bvand", other(), ctx.const(255, 256))
                nxt = mk(r.choice(["bvshl", "bvlshr", "bvashr"]), prev, sh)
            elif kind == "cmp":
                bools.append(mk(r.choice(["bvult", "bvule", "bvslt", "="]), prev, other()))
                continue
            elif kind == "ite":
                c = bools.pop() if bools else mk("bvult", prev, other())
                nxt = mk("ite", c, prev, other())
            elif kind == "struct":
                lo = r.randrange(0, 128)
                hi_part = mk("extract", prev, params=(lo + 127, lo))
                o = other()
                lo_part = mk("extract", o, params=(127, 0))
                nxt = mk("concat", hi_part, lo_part) if r.random() < 0.6 else mk("zero_extend", hi_part, params=(128,))
            else:  # div
                nxt = mk(r.choice(["bvudiv", "bvurem"]), prev, mk("bvor", other(), ctx.const(1, 256)))
            prev = nxt
            recent.append(nxt)
        ends.append(prev)
        pend_bools.append(bools)
    return ctx, leaves, ends, pend_bools, count


def build_c5(evaluate: Callable[[Sequence[Node], int, int], List[int]], n_nodes: int = 10000,
             n_leaves: int = 16, n_conj: int = 32, seed: int = 0x5EED0005,
             witness_index: int = 0x5EED0005 % (1 << 31), density_log2: int = 24,
             keep_pending: bool = True) -> Synthetic:
    """evaluate(terms, candidate_index, seed) -> values of `terms` at that candidate.

    keep_pending=False drops the chains' leftover comparisons (each halves the
    satisfying density), so density_log2 alone sets it: the mixed-verdict
    variant of the full-size parity test (tests/test_gpu_fullsize.py)."""
    ctx, leaves, ends, pend, count = build_chains(n_nodes, n_leaves, n_conj, seed)
    vals = evaluate(ends, witness_index, seed)
    pend_vals = evaluate([b for bs in pend for b in bs], witness_index, seed) if any(pend) else []
    frac = 2.0 ** (-density_log2 / n_conj)
    conj: List[Node] = []
    k = 0
    for e, v, bs in zip(ends, vals, pend):
        t = max(v + 1, int(frac * (1 << 256)))
        t = min(t, M256)
        c = ctx.app("bvult", e, ctx.const(t, 256))
        # leftover comparisons stay reachable: AND them in with the polarity they have at the witness
        for b in bs:
            bv = pend_vals[k]
            k += 1
            if keep_pending:
                c = ctx.app("and", c, b if bv else ctx.app("not", b))
        conj.append(c)
    return Synthetic(ctx, leaves, ends, conj, witness_index, seed, count + len(conj))
