"""Replay ``--solver-log`` dumps through the witness engine.

``myth analyze --solver-log DIR`` writes every uncached query as the SMT-LIB2
text of z3's ``Optimize.sexpr()`` (mythril/support/model.py:45-56).  This
module parses such files (mythril_amd/smt2.py), routes them the way the
drop-in ``get_model`` does — queries with ``minimize``/``maximize`` stay with z3,
formulas outside the vocabulary fall back — and searches the rest on the
device, many programs per launch.  It gives offline replays and benchmarks of
real analyses without z3 or solc.

    python -m mythril_amd.replay DIR [--budget 2^22] [--batch 64]
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time
from dataclasses import dataclass, field
from typing import List, Optional

from .compiler import Unsupported


@dataclass
class Result:
    path: str
    status: str                      # "witness" | "miss" | "z3" (objectives) | "unsupported"
    index: Optional[int] = None
    values: dict = field(default_factory=dict)
    reason: str = ""
    arrays: dict = field(default_factory=dict)      # array -> {index: value} (Ackermann leaves)
    functions: dict = field(default_factory=dict)   # UF -> {args: value}


def load(path: str):
    from .engine import prepare
    from .smt2 import parse_file
    s = parse_file(path)
    if s.minimize or s.maximize:
        return s, None, "objectives: answered by z3 (analysis/solver.py:51-101)"
    return s, prepare(s.asserts, s.ctx), ""


def replay(paths: List[str], engine, batch: int = 64) -> List[Result]:
    out: List[Result] = []
    pending = []
    for p in paths:
        try:
            s, q, why = load(p)
        except (Unsupported, RecursionError, ValueError, KeyError) as e:
            out.append(Result(p, "unsupported", reason=str(e)))
            continue
        if q is None:
            out.append(Result(p, "z3", reason=why))
            continue
        pending.append((p, s, q))
    for i in range(0, len(pending), batch):
        chunk = pending[i:i + batch]
        found = engine.search([q for _, _, q in chunk])
        for (p, s, q), w in zip(chunk, found):
            if w is None:
                out.append(Result(p, "miss"))
            else:
                out.append(Result(p, "witness", w.index, dict(w.values), arrays=w.arrays, functions=w.functions))
    order = {p: k for k, p in enumerate(paths)}
    return sorted(out, key=lambda r: order[r.path])


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("paths", nargs="+", help=".smt2 files or directories")
    ap.add_argument("--budget", type=int, default=1 << 22, help="candidates per query")
    ap.add_argument("--batch", type=int, default=64, help="programs per launch")
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args(argv)
    files = []
    for p in a.paths:
        files += sorted(glob.glob(os.path.join(p, "*.smt2")) + glob.glob(os.path.join(p, "*.smt2.gz"))) \
            if os.path.isdir(p) else [p]
    from .engine import WitnessEngine
    eng = WitnessEngine(device=a.device, budget=a.budget)
    t0 = time.perf_counter()
    res = replay(files, eng, a.batch)
    dt = time.perf_counter() - t0
    for r in res:
        print(json.dumps({"file": os.path.basename(r.path), "status": r.status, "index": r.index,
                          "reason": r.reason}))
    summary = {k: sum(1 for r in res if r.status == k) for k in ("witness", "miss", "z3", "unsupported")}
    print(json.dumps({"files": len(res), **summary, "seconds": dt, "engine": eng.stats}), flush=True)
    eng.close()


if __name__ == "__main__":
    sys.exit(main())
