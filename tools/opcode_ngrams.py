#!/usr/bin/env python3
"""Opcode sequences of the committed corpora (tests/golden/laser and
solver_log), for the asm interpreter's fused handlers (mythril_amd/isa.py
ASM_FUSED): each query's program is weighted equally, and sequences of 2-4
opcodes are picked greedily by the dispatches they save when every program is
tokenised left to right, longest match first (as mw_asm_predecode does).

    python tools/opcode_ngrams.py [--n 24] [--out profiles/.../opcode_ngrams.json]
"""
import argparse
import collections
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

# handlers that take the next instructions themselves (W_CDINS chains) or end
# the program never join a fused sequence
NEVER = {"W_CDINS", "END"}


def programs():
    from mythril_amd import isa
    from mythril_amd.engine import prepare
    from mythril_amd.smt2 import parse_file
    names = {c: n for n, c in isa.OPCODES.items()}
    out = []
    for corpus in ("laser", "solver_log"):
        for f in sorted(glob.glob(os.path.join(ROOT, "tests", "golden", corpus, "*.smt2*"))):
            s = parse_file(f)
            try:
                q = prepare(s.asserts, s.ctx)
            except Exception:   # noqa: BLE001 - unsupported queries have no program
                continue
            code = list(q.program.code)
            ops = [names.get(int(w) & 0xFF, "?") for w in code[0::4]]
            if isa.asm_eligible(q.program.code, q.program.leaves, q.program.consts):
                out.append((corpus, ops))
    return out


def tokenise(ops, fused):
    """dispatches of one program under the fused set (longest match first)"""
    by_len = sorted(fused, key=len, reverse=True)
    i, n = 0, 0
    while i < len(ops):
        for t in by_len:
            if tuple(ops[i:i + len(t)]) == t:
                i += len(t)
                break
        else:
            i += 1
        n += 1
    return n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=24)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    progs = programs()
    weights = [1.0 / len(ops) for _, ops in progs]
    total = sum(len(ops) * w for (_, ops), w in zip(progs, weights))
    fused = []
    log = []
    for _ in range(a.n):
        cand = collections.Counter()
        for (_, ops), w in zip(progs, weights):
            for L in (2, 3, 4):
                for i in range(len(ops) - L + 1):
                    t = tuple(ops[i:i + L])
                    if not NEVER.intersection(t):
                        cand[t] += w
        base = sum(tokenise(ops, fused) * w for (_, ops), w in zip(progs, weights))
        best, gain = None, 0.0
        for t, _ in cand.most_common(60):
            g = base - sum(tokenise(ops, fused + [t]) * w for (_, ops), w in zip(progs, weights))
            if g > gain:
                best, gain = t, g
        if best is None:
            break
        fused.append(best)
        log.append({"seq": list(best), "dispatches_saved": round(gain / total, 4)})
        print(f"{' '.join(best):45s} saves {gain / total:6.3f} of all dispatches")
    after = sum(tokenise(ops, fused) * w for (_, ops), w in zip(progs, weights))
    print(f"dispatches: {after / total:.3f} of the instructions ({len(progs)} programs)")
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"programs": len(progs), "dispatch_fraction": after / total, "picked": log}, f, indent=1)


if __name__ == "__main__":
    main()
