"""Throughput of the C2-C4 solver-log queries (BASELINE.json configs[1..3]).

C2: token.sol -t 3 transfer queries, 2^24 candidates each;
C3: BECToken batchTransfer SWC-101 overflow query, 2^28 candidates;
C4: WalletLibrary -t 3 queries searched together in one launch (state
    batching), 2^24 candidates;
C2L: the LASER-shaped queries of token.sol's runtime bytecode
    (tests/golden/laser/underflow_*, from the reference's underflow.sol.o),
    all in one launch, 2^24 candidates each.

The queries are the committed ``--solver-log``-format dumps
(tests/golden/solver_log, synthetic: no z3/solc exists to dump real ones, see
tests/make_solver_log_corpus.py).  Each config is timed twice in exhaustive
mode (early exit off): the threaded-dispatch asm interpreter (the default for
these programs), the compiled interpreter (MYTHRIL_AMD_ASM=0) and the
specialised kernel (mythril_amd/jit.py).  Time to first witness (early exit + stop-after-hit,
interpreter) is reported beside it.  evals/s = programs x candidates / wall
time of the mg_search call; the roofline uses the kernel time from the library's
HIP events.  Two op counts are reported: the compiler's ops_per_eval (SURVEY.md
§8(d) priced on the lowered DAG) and executed_ops_per_eval (the same units
priced per instruction of the program the engine runs, isa.insn_ops: a
congruence grid row is one table lookup, not the n pair checks the DAG
states).  frac_peak uses the smaller of the two, so no
engine claims more work than its instructions execute; frac_peak_nominal
keeps the DAG count.  The hipcc-specialised tier compiles the unfused SSA
(no grids): its executed count is the DAG's.

    python tools/config_bench.py [--out FILE] [--no-jit]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

LOG = os.path.join(ROOT, "tests", "golden", "solver_log")
LASER = os.path.join(ROOT, "tests", "golden", "laser")
CONFIGS = [
    ("C2", ["c2_token_transfer_ok.smt2", "c2_token_transfer_underflow.smt2"], 24, False),
    # C2 on queries derived from the reference's own bytecode: every JUMPI
    # successor set of a 2-3 transaction token.sol run (underflow.sol.o),
    # searched together in one launch (LaserEVM batching)
    ("C2L", sorted(f for f in os.listdir(LASER) if f.startswith("underflow_") and f.endswith(".smt2.gz")), 24, True),
    ("C3", ["c3_bec_batchtransfer_overflow.smt2"], 28, False),
    ("C4", ["c4_wallet_onlyowner.smt2", "c4_wallet_contradiction.smt2"], 24, True),
]
SLICE = 1 << 24   # candidates per launch


def _groups(files, together):
    from mythril_amd.engine import prepare
    from mythril_amd.smt2 import parse_file
    qs = []
    for f in files:
        s = parse_file(os.path.join(LASER if f.endswith(".gz") else LOG, f))
        qs.append(prepare(s.asserts, s.ctx))
    return [(files, qs)] if together else [([f], [q]) for f, q in zip(files, qs)]


def warm_jobs():
    """One compile job per query group (independent hipcc runs; tools/jit_warm.py
    runs them in parallel).  The queries are prepared here, in the caller's thread."""
    from mythril_amd import jit
    jobs = []
    for _, files, _, together in CONFIGS:
        for _, g in _groups(files, together):
            progs = [q.program for q in g]
            jobs.append(lambda progs=progs: jit.compile_device(progs, "xe", waves=2, lds_leaves=0))
    return jobs


def warm():
    """Compile the specialised kernels into build/jit (CPU)."""
    for job in warm_jobs():
        job()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--no-jit", action="store_true")
    ap.add_argument("--warm", action="store_true", help="only compile the specialised kernels into build/jit (CPU)")
    ap.add_argument("--only", default=None, help="comma-separated config names (default: all)")
    ap.add_argument("--engines", default=None, help="comma-separated engines (default: asm,asmjit,interp[,jit])")
    a = ap.parse_args()
    import bench
    from mythril_amd import isa, jit
    from mythril_amd.engine import DEFAULT_SEED
    from mythril_amd.runtime import Device
    if a.warm:
        warm()
        return
    dev = Device(0)
    peak = bench.THEORETICAL_PEAK
    lines = []
    for name, files, log2, together in CONFIGS:
        if a.only and name not in a.only.split(","):
            continue
        for gfiles, g in _groups(files, together):
            # the program a search of this length runs (engine.search_program:
            # the quarter layout's compile when the work repays it)
            from mythril_amd.engine import search_program
            dps = [dev.load(search_program(q, 1 << log2)) for q in g]
            ops = sum(q.ops_per_eval for q in g)
            exec_ops = sum(isa.executed_ops_per_eval(dp.prog.code) for dp in dps)
            count = 1 << log2
            # time to first witness (interpreter, early exit)
            t0 = time.perf_counter()
            first = [None] * len(dps)
            pos = 0
            while pos < count and any(x is None for x in first):
                found, _ = dev.search(dps, DEFAULT_SEED, pos, min(SLICE, count - pos),
                                      isa.FLAG_EARLY_EXIT | isa.FLAG_STOP_AFTER_HIT)
                first = [x if x is not None else y for x, y in zip(first, found)]
                pos += SLICE
            ttfw = time.perf_counter() - t0
            engines = ["asm", "asmjit", "interp"] if a.no_jit else ["asm", "asmjit", "interp", "jit"]
            if a.engines:
                engines = a.engines.split(",")
            for engine in engines:
                compile_s = None
                # asm: the threaded-dispatch interpreter (the default for these
                # programs); asmjit: each program's assembled kernel
                # (mythril_amd/asmjit.py, attached here, assembly time reported);
                # interp: the compiled interpreter (MYTHRIL_AMD_ASM=0, which also
                # turns the assembled kernels off); jit: hipcc's specialised kernel
                os.environ["MYTHRIL_AMD_ASM"] = "0" if engine == "interp" else "1"
                if engine == "asmjit":
                    from mythril_amd import asmjit
                    compile_s = sum(asmjit.attach(dev, dp, cache=False) for dp in dps)
                if engine == "jit":
                    compile_s = jit.attach(dev, dps, variants="xe", waves=2, lds_leaves=0)
                ran = sorted({dev.engine_of(dp) for dp in dps})
                dev.search(dps, DEFAULT_SEED, 0, SLICE, 0)            # warm-up
                kms, evals = 0.0, 0
                t0 = time.perf_counter()
                for pos in range(0, count, SLICE):
                    _, st = dev.search(dps, DEFAULT_SEED, pos, SLICE, 0)
                    kms += st["kernel_ms"]
                    evals += st["evals"]
                wall = time.perf_counter() - t0
                nominal = ops * count / (kms / 1e3)
                ex = ops if engine == "jit" else exec_ops      # hipcc compiles the unfused SSA
                achieved = min(ops, ex) * count / (kms / 1e3)
                line = {"config": name, "files": gfiles, "engine": engine + (f" ({dps[0].kernel})" if dps[0].kernel else ""),
                        "kernels": ran,
                        "programs": len(g), "candidates": count, "evals": evals,
                        "evals_per_s": len(g) * count / wall, "kernel_ms": kms, "ops_per_eval": ops,
                        "executed_ops_per_eval": ex,
                        "tops": achieved / 1e12, "frac_peak": achieved / peak, "frac_peak_nominal": nominal / peak,
                        "jit_compile_s": compile_s, "first_witness": first, "ttfw_s": ttfw}
                print(json.dumps(line), flush=True)
                lines.append(line)
            for dp in dps:
                dp.free()
    dev.close()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(lines, f, indent=1)


if __name__ == "__main__":
    main()
