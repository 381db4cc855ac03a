#!/usr/bin/env python3
"""Structural UNSAT arguments for the corpus queries no search witnessed
(TEST INFRASTRUCTURE, CPU only).

tools/ground_truth.py searches every "unknown" query of tests/golden/laser up
to 2^32 candidates on the device; what it leaves without a witness is listed
in its JSON.  Without z3 (absent here and on the box) nothing proves those
UNSAT in general, so each one gets the reason this script can give, from the
lowered formula (engine.prepare: `If(c,1,0) = 0` folded to `not c`, arrays and
UFs Ackermannised):

  propagation   unit propagation over top-level facts `v = K` (and `v = w`)
                fixes variables until some conjunct evaluates to false
                (the oracle's evaluator, oracle/dag_eval.py): e.g.
                MutationPruner's `call_value > 0` on a path that checked
                `call_value = 0` (a non-payable function);
  interval      the unsigned bounds a variable gets from top-level
                comparisons with constants are empty;
  tautology     a conjunct folds to false once `x <u 0` (never) and
                `x >=u 0` (always) are folded, as solc 0.4's `a - b >= 0`
                underflow checks on uints make them;
  open          neither applies (the reason is argued by hand in DESIGN.md).

    python tools/unsat_proofs.py GROUND_TRUTH.json [--out FILE]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from mythril_amd.compiler import _flatten  # noqa: E402
from mythril_amd.engine import prepare  # noqa: E402
from mythril_amd.ir import BOOL, free_vars  # noqa: E402
from mythril_amd.smt2 import parse_file  # noqa: E402
from oracle.dag_eval import eval_nodes  # noqa: E402

CORPUS = os.path.join(ROOT, "tests", "golden", "laser")
_CMP = {"bvult", "bvule", "bvugt", "bvuge"}


def _facts(conj):
    """(var name -> value) from top-level v = K, and v = w equalities."""
    fixed, same = {}, []
    for c in conj:
        if c.op == "=" and len(c.args) == 2:
            a, b = c.args
            if a.op == "const":
                a, b = b, a
            if a.op == "var" and b.op == "const" and a.width != BOOL:
                fixed[a.name] = b.val
            elif a.op == "var" and b.op == "var":
                same.append((a.name, b.name))
        elif c.op == "var" and c.width == BOOL:
            fixed[c.name] = 1
        elif c.op == "not" and c.args[0].op == "var":
            fixed[c.args[0].name] = 0
    changed = True
    while changed:
        changed = False
        for x, y in same:
            for p, q in ((x, y), (y, x)):
                if p in fixed and q not in fixed:
                    fixed[q] = fixed[p]
                    changed = True
    return fixed


_NEVER = {"bvult": (1, 0), "bvugt": (0, 0)}     # x <u 0 and 0 >u x: false
_ALWAYS = {"bvuge": (1, 0), "bvule": (0, 0)}    # x >=u 0 and 0 <=u x: true


def tautology(conj, ctx):
    """Fold the comparisons with 0 that hold or fail for every value (x <u 0,
    x >=u 0: the unsigned underflow checks `a - b >= 0` of solc 0.4 code) and
    then every constant subterm (the oracle's evaluator); a conjunct that folds
    to false makes the set UNSAT."""
    from oracle.dag_eval import _eval1
    from mythril_amd.ir import topo
    memo = {}
    for n in topo(conj):
        args = [memo[a.id] for a in n.args]
        r = None
        if n.op in _NEVER or n.op in _ALWAYS:
            side, val = _NEVER.get(n.op) or _ALWAYS.get(n.op)
            k = args[side]
            if k.op == "const" and k.val == val:
                r = ctx.const(0 if n.op in _NEVER else 1, BOOL)
        if r is None and args and all(a.op == "const" for a in args) and n.op not in ("select", "store", "apply"):
            try:
                v = _eval1(n, [a.val for a in args], {})
                r = ctx.const(v, n.width)
            except Exception:   # noqa: BLE001 - not foldable here
                r = None
        if r is None:
            r = n if all(a is b for a, b in zip(args, n.args)) else ctx._mk(n.op, n.width, tuple(args), n.params,
                                                                          n.val, n.name, n.dom)
        memo[n.id] = r
    for i, c in enumerate(conj):
        f = memo[c.id]
        if f.op == "const" and not f.val:
            return {"reason": "tautology", "false_conjunct": i}
    return None


def propagation(conj):
    fixed = _facts(conj)
    if not fixed:
        return None
    for i, c in enumerate(conj):
        vs = [v for v in free_vars([c]) if v.op == "var"]
        if vs and all(v.name in fixed for v in vs):
            if not eval_nodes([c], dict(fixed))[c.id]:
                return {"reason": "propagation", "false_conjunct": i,
                        "fixed": sorted(v.name for v in vs)}
    return None


def interval(conj):
    lo, hi = {}, {}
    for c in conj:
        neg = c.op == "not"
        t = c.args[0] if neg else c
        if t.op not in _CMP or len(t.args) != 2:
            continue
        a, b = t.args
        op = t.op
        if a.op == "const" and b.op == "var":
            a, b = b, a
            op = {"bvult": "bvugt", "bvugt": "bvult", "bvule": "bvuge", "bvuge": "bvule"}[op]
        if not (a.op == "var" and b.op == "const"):
            continue
        if neg:
            op = {"bvult": "bvuge", "bvuge": "bvult", "bvule": "bvugt", "bvugt": "bvule"}[op]
        k, n = b.val, a.name
        top = (1 << a.width) - 1
        if op == "bvult":
            hi[n] = min(hi.get(n, top), k - 1)
        elif op == "bvule":
            hi[n] = min(hi.get(n, top), k)
        elif op == "bvugt":
            lo[n] = max(lo.get(n, 0), k + 1)
        else:
            lo[n] = max(lo.get(n, 0), k)
    for n in set(lo) & set(hi):
        if lo[n] > hi[n]:
            return {"reason": "interval", "var": n, "lo": hex(lo[n]), "hi": hex(hi[n])}
    for n, h in hi.items():
        if h < 0:
            return {"reason": "interval", "var": n, "lo": "0x0", "hi": str(h)}
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("ground_truth")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    gt = json.load(open(a.ground_truth))
    man = {m["file"]: m for m in json.load(open(os.path.join(CORPUS, "manifest.json")))}
    out = {}
    for f in gt["no_witness"]:
        s = parse_file(os.path.join(CORPUS, f))
        q = prepare(s.asserts, s.ctx)
        conj = _flatten(q.lowered.conjuncts)
        why = propagation(conj) or interval(conj) or tautology(conj, q.ctx) or {"reason": "open"}
        why["kind"] = man[f]["kind"]
        out[f] = why
    counts = {}
    for w in out.values():
        counts[w["reason"]] = counts.get(w["reason"], 0) + 1
    print(json.dumps(counts))
    for f, w in out.items():
        if w["reason"] == "open":
            print("open:", f, w["kind"])
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
