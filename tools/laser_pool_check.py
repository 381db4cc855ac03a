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
    """{leaf name: model value} for the program's leaves.  Array reads and UF
    applications are resolved in rounds: an argument term may itself read an
    earlier Ackermann leaf (keccak of a keccak), whose value joins the model
    before the next round."""
    low = q.lowered
    out = {}
    m = dict(model)
    pending = dict(low.ack)
    for _ in range(len(pending) + 1):
        progress = False
        for name, al in list(pending.items()):
            try:
                vals = eval_nodes(list(al.args), m)
            except KeyError:
                continue
            args = tuple(vals[a.id] for a in al.args)
            base = model.get(al.base)
            if al.kind == "select":
                v = base.get(args[0]) if base is not None else None
            else:
                d, default = base if base is not None else ({}, 0)
                v = d.get(args, default)
            m[name] = v
            del pending[name]
            progress = True
        if not progress:
            break
    for node in q.program.leaf_nodes:
        base, _, chunk = node.name.partition("#")   # >256-bit leaves: 256-bit chunk k
        v = m.get(base)
        if isinstance(v, int) and chunk:
            v = (v >> (256 * int(chunk))) & ((1 << 256) - 1)
        out[node.name] = v if isinstance(v, int) else None
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
    ap.add_argument("--only", default=None, help="comma-separated query files")
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
                if status.get(fn) != "sat" or (a.only and fn not in a.only.split(",")):
                    continue
                q = prepare(rq.constraints, m.c)
                missing, broken = check(q, run.model)
                if missing or broken or a.all:
                    report.append({"file": fn, "uncovered": missing, "broken_ties": broken})
                    print(json.dumps(report[-1]), flush=True)
    print(f"{len(report)} SAT queries with uncovered leaves")


if __name__ == "__main__":
    main()
