#!/usr/bin/env python3
"""Which SAT LASER queries (tests/golden/laser) cannot be witnessed from the
pools alone.

For every SAT query the concolic run's model (tests/laser_concolic.py,
re-run per scenario) gives each program leaf its value: a plain variable by
name, an array read / UF application by evaluating its index or argument terms
under the model.  A leaf is COVERED when its value is a (non-RANDOM) entry of
its pool; tied calldata bytes must share one entry index.  Uncovered leaves
can only be hit by a RANDOM draw (2^-8 per byte, 2^-256 per word).

    python tools/laser_pool_check.py [--all]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from make_laser_corpus import SCENARIOS, load_code  # noqa: E402
from mythril_amd.engine import prepare  # noqa: E402
from oracle.dag_eval import eval_nodes  # noqa: E402
from tests.laser_concolic import ACTORS, run_sequence  # noqa: E402


def leaf_values(q, model):
    """{leaf name: model value} for the program's leaves."""
    low = q.lowered
    out = {}
    arg_terms = []
    for al in low.ack.values():
        arg_terms.extend(al.args)
    vals = eval_nodes(list(q.conjuncts) + arg_terms, model) if arg_terms else {}
    for node in q.program.leaf_nodes:
        name = node.name
        al = low.ack.get(name.split("#")[0])
        if al is None:
            v = model.get(name)
            out[name] = v if isinstance(v, int) else None
            continue
        args = tuple(vals.get(a.id) if a.op != "const" else a.val for a in al.args)
        base = model.get(al.base)
        if al.kind == "select":
            out[name] = base.get(args[0]) if base is not None else None
        else:
            d, default = base if base is not None else ({}, 0)
            out[name] = d.get(args, default)
    return out


def check(q, model):
    vals = leaf_values(q, model)
    specs = {s.name: s for s in q.program.leaf_specs}
    missing = []
    ties = {}
    for name, v in vals.items():
        sp = specs.get(name)
        if v is None or sp is None or sp.pool is None:
            continue
        idx = [i for i, e in enumerate(sp.pool) if e is not None and e == v & ((1 << sp.width) - 1)]
        if not idx:
            missing.append((name, hex(v), len(sp.pool), sum(e is None for e in sp.pool)))
        lead = sp.tie or (name if any(s.tie == name for s in specs.values()) else None)
        if lead:
            ties.setdefault(lead, []).append(set(idx))
    broken = [lead for lead, sets in ties.items() if sets and not set.intersection(*sets)]
    return missing, broken


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--all", action="store_true", help="report covered queries too")
    a = ap.parse_args()
    manifest = json.load(open(os.path.join(ROOT, "tests", "golden", "laser", "manifest.json")))
    status = {m["file"]: m["status"] for m in manifest}
    report = []
    for contract, scenarios in SCENARIOS.items():
        code = load_code(contract)
        for name, txs in scenarios:
            m, run = run_sequence(code, txs, balances={x: 10 ** 18 for x in ACTORS.values()})
            for qi, rq in enumerate(run.queries):
                fn = f"{contract}_{name}_q{qi:02d}_{'sat' if rq.sat else 'unknown'}.smt2.gz"
                if status.get(fn) != "sat":
                    continue
                q = prepare(rq.constraints, m.c)
                missing, broken = check(q, run.model)
                if missing or broken or a.all:
                    report.append({"file": fn, "uncovered": missing, "broken_ties": broken})
                    print(json.dumps(report[-1]), flush=True)
    print(f"{len(report)} SAT queries with uncovered leaves")


if __name__ == "__main__":
    main()
