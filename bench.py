#!/usr/bin/env python3
"""Benchmark: candidate-assignment evals/sec of the witness search (BASELINE.json).

Workload (BASELINE.json config C5, the metric's multi-GPU config): a synthetic
10k-node 256-bit bitvector DAG over 16 free 256-bit variables whose root is
the AND of 32 comparisons with a planted witness (mythril_amd/synth.py).  A
step is one exhaustive search launch over a batch of candidate indices per GPU
(early exit off, so every verdict is fully determined — SURVEY.md §8(d)).
Candidates are generated on the device from the index (Philox4x32-10); the
program is uploaded once before timing.

Multi-GPU: one process per GPU; rank r searches its own contiguous slice of
the index space each step (weak scaling, no data-path collective); the witness
minimum is combined with one RCCL all-reduce(MIN) of a single int64, as the
engine's multi-GPU search does (mythril_amd/distributed.py).  Ranks come from
torchrun (WORLD_SIZE set: it must equal --gpus), or, when `--gpus N` is given
without a torchrun environment, from N rank processes this script starts
itself before anything here touches a GPU (launch_ranks).

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# CDNA4 issues a wave64 VALU instruction in 2 cycles on a 32-lane SIMD
# (MI355X_MICROARCH.md): 256 CU x 4 SIMD x 32 lanes x 2.4 GHz
THEORETICAL_PEAK = 256 * 4 * 32 * 2.4e9
BENCH_VARIANTS = "x"  # exhaustive kernel only: the bench never exits early
BENCH_WAVES = 2  # with 10 leaves in LDS (profiles/r1_v4_jit); 1 wave/SIMD: 512 registers, no LDS
BENCH_INTERLEAVE = 1  # conjunct streams merged per basic block (jit.interleave_conjuncts)
BENCH_SPLIT = False  # one kernel: 111.7M evals/s; as 5 part kernels (split_ssa): 109.9M, 7x faster to compile


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs, one rank process each (default: WORLD_SIZE under torchrun, else 1); without a "
                         "torchrun environment N > 1 starts the N ranks itself")
    ap.add_argument("--begin", type=int, default=0, help="first candidate index of warmup step 0")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL over xGMI) on GPUs; gloo only with --host-emulator (CPU tests)")
    # CPU tests of the rank plumbing: the host build of the interpreter stands in
    # for the device (tests/fakedev.py); never a product or benchmark path
    ap.add_argument("--host-emulator", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch-log2", type=int, default=22, help="candidates per GPU per step = 2**k")
    ap.add_argument("--nodes", type=int, default=10000)
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ttfw", action="store_true", help="skip the time-to-first-witness search")
    ap.add_argument("--no-recount", action="store_true",
                    help="skip the untimed counting pass (profiling runs: every dispatch of the kernel is then a "
                         "timed-form launch; the division-path counts and the executed roofline are not reported)")
    ap.add_argument("--ttfw-slice-log2", type=int, default=24, help="candidates per rank per stop-after-hit slice")
    ap.add_argument("--ttfw-max-slices", type=int, default=128)
    ap.add_argument("--ttfw-begin", type=int, default=0, help="first index of the time-to-first-witness sweep")
    ap.add_argument("--engine", choices=["jit", "interp"], default="jit",
                    help="jit: the program's specialised straight-line kernel (mythril_amd/jit.py); "
                         "interp: the bytecode interpreter")
    ap.add_argument("--jit-waves", type=int, default=BENCH_WAVES, choices=[1, 2, 3, 4],
                    help="waves per SIMD the specialised kernel is built for")
    ap.add_argument("--jit-split", type=int, default=int(BENCH_SPLIT), choices=[0, 1],
                    help="1: split the program into part kernels at conjunct boundaries")
    ap.add_argument("--devices", type=int, default=1,
                    help="single-process multi-GPU (mythril_amd/multidev.py): this process drives N devices, "
                         "each searching its slice of every step (the torchrun path is the default)")
    ap.add_argument("--jit-interleave", type=int, default=BENCH_INTERLEAVE,
                    help="conjuncts interleaved per instruction stream in the specialised kernel")
    ap.add_argument("--jit-lds-leaves", type=int, default=None,
                    help="leaves kept in LDS instead of registers (default: 10 at 2 waves/SIMD, 0 at 1)")
    return ap.parse_args()


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` without torchrun: start N rank processes (this same
    script with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, as torchrun
    would) and return the first failing exit code.  The parent never touches a
    GPU (no HIP call, no torch.cuda), so nothing is exec'd from a process that
    initialised one.  If a rank fails the others are stopped, so a dead peer
    cannot leave them waiting in a collective."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None:
        world = args.gpus or 1
        if world > 1:
            sys.exit(launch_ranks(world))
    else:
        world = int(world_env)
        if args.gpus is not None and args.gpus != world:
            raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.devices > 1 and world > 1:
        # both would split the same candidates over overlapping GPUs
        raise SystemExit("bench.py: --devices (one process, N GPUs) and ranks (one process per GPU) exclude each other")
    if args.dist_backend == "gloo" and not args.host_emulator:
        raise SystemExit("bench.py: gloo is for --host-emulator CPU tests; GPUs use nccl (RCCL)")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    coll_dev = "cpu" if args.host_emulator else f"cuda:{local}"
    if world > 1:
        import torch
        import torch.distributed as dist
        if not args.host_emulator:
            torch.cuda.set_device(local)
        dist.init_process_group(args.dist_backend, rank=rank, world_size=world)

    from mythril_amd.compiler import compile_program
    from mythril_amd.runtime import unpack_trace
    from mythril_amd.synth import build_c5

    if args.host_emulator:
        from tests.fakedev import FakeDevice
        dev = FakeDevice(chunk=1 << 12)
        if args.engine != "interp":
            raise SystemExit("bench.py: --host-emulator runs the interpreter only")
    else:
        from mythril_amd.runtime import Device
        dev = Device(local)
    multi = None
    if args.devices > 1:
        from mythril_amd.multidev import MultiDevice
        multi = MultiDevice([dev] + [Device(i) for i in range(1, args.devices)])

    def gpu_eval(terms, index, seed):
        p = compile_program([], trace=list(terms))
        dp = dev.load(p)
        _, tr = dev.eval_generated(dp, seed, index, 1)
        dp.free()
        return [unpack_trace(p, tr, t)[0] for t in terms]

    syn = build_c5(gpu_eval, n_nodes=args.nodes)
    prog = compile_program(syn.conjuncts)
    dp = dev.load(prog)
    mdp = multi.load(prog) if multi is not None else None
    jit_s = None
    if args.engine == "jit":
        # one-time program preparation, like the upload: outside the timed region
        # (the in-tree cache, warmed by __graft_entry__.build(), usually makes it 0)
        from mythril_amd import jit
        if args.jit_lds_leaves is None:  # LDS: waves/SIMD x slots x 8 KiB per CU <= 160 KiB
            args.jit_lds_leaves = {1: 0, 2: jit.BENCH_LDS_LEAVES, 3: 6, 4: 5}[args.jit_waves]
        split = bool(args.jit_split)
        if not split and not jit.is_cached([prog], BENCH_VARIANTS, args.jit_waves, args.jit_lds_leaves,
                                           args.jit_interleave):
            # one kernel compiles for ~6 min; its parts in ~1 min (parallel hipcc)
            print("[bench] single-kernel code object not cached: using the split kernels", file=sys.stderr)
            split = True
        args.jit_split = int(split)
        jit_s = jit.attach(dev, [dp], variants=BENCH_VARIANTS, waves=args.jit_waves, lds_leaves=args.jit_lds_leaves,
                           split=split, interleave=args.jit_interleave)
        if multi is not None:
            for d, part in zip(multi.devs[1:], mdp.parts[1:]):
                jit.attach(d, [part], variants=BENCH_VARIANTS, waves=args.jit_waves,
                           lds_leaves=args.jit_lds_leaves, split=split, interleave=args.jit_interleave)
            mdp.parts[0].free()
            mdp.parts[0] = dp   # device 0's copy is the program the kernel was attached to above
    batch = 1 << args.batch_log2
    from mythril_amd import isa
    # The timed launches write no launch counters (isa.FLAG_NO_COUNT: the
    # specialised kernel's per-wave atomics were 11 MiB of HBM writes per
    # launch, profiles/pmc_traffic.json r4ad); the same steps run again after
    # the timed region with the counters on, for the division-path counts the
    # executed-work roofline is priced from.
    TIMED_FLAGS = isa.FLAG_NO_COUNT

    def step(k, flags=0):
        if multi is not None:   # one process: every device searches its slice of the step
            begin = (args.begin + k * args.devices * batch) % (1 << 62)
            (found,), st = multi.search([mdp], syn.seed, begin, batch * args.devices, flags)
            return found, st
        begin = (args.begin + (k * world + rank) * batch) % (1 << 62)
        (found,), st = dev.search([dp], syn.seed, begin, batch, flags)
        return found, st

    for k in range(args.warmup):
        step(k, TIMED_FLAGS)

    def barrier():
        if dist is not None:
            import torch
            t = torch.zeros(1, device=coll_dev)
            dist.all_reduce(t)
            if not args.host_emulator:
                torch.cuda.synchronize()

    barrier()
    kms = []
    dcounts = []
    found_any = None
    t0 = time.perf_counter()
    timed_evals = 0
    for k in range(args.warmup, args.warmup + args.steps):
        found, st = step(k, TIMED_FLAGS)
        kms.append(st.get("kernel_ms", 0.0))
        timed_evals += st.get("evals", 0)
        if found is not None:
            found_any = found if found_any is None else min(found_any, found)
    barrier()
    elapsed = time.perf_counter() - t0
    # the counting pass (untimed): the same K launches with the counters on
    recount = found_any if args.no_recount else None
    for k in (range(args.warmup, args.warmup + args.steps) if not args.no_recount else ()):
        found, st = step(k, 0)
        dcounts.append(st)
        if found is not None:
            recount = found if recount is None else min(recount, found)
    if recount != found_any:
        print(f"[bench] PARITY FAILURE: the counting pass found {recount}, the timed launches {found_any}",
              file=sys.stderr)
    rccl_world = 1
    if dist is not None:
        import torch
        rccl_world = dist.get_world_size()
        t = torch.tensor([elapsed], dtype=torch.float64, device=coll_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        from mythril_amd.distributed import allreduce_min
        (found_any,) = allreduce_min([found_any], device=coll_dev)  # RCCL MIN of the witness index

    total_evals = world * args.steps * batch * max(1, args.devices)
    value = total_evals / elapsed
    avg_kernel_s = sum(kms) / len(kms) / 1e3
    # executed algorithmic work per launch: every wide division priced by the
    # path each wave took (mg_stats.lane_div_*; compiler.DIV_PRICE_*), and the
    # division-free floor beside it
    from mythril_amd.multidev import DIV_COUNTS
    per_launch = {k: sum(st.get(k, 0) for st in dcounts) / max(1, len(dcounts)) / max(1, args.devices)
                  for k in DIV_COUNTS}
    ops_launch = prog.executed_ops(batch, per_launch)
    ops_floor = prog.executed_ops(batch, None)
    achieved = ops_launch / avg_kernel_s if avg_kernel_s > 0 else 0.0
    measured_peak = load_measured_peak()

    # time to first witness: every rank searches its share of each slice, and
    # one all-reduce(MIN) per slice stops all of them at the first slice with a
    # hit (the cross-rank early stop of SURVEY.md §8(e))
    ttfw = None if args.no_ttfw else time_to_first_witness(dev, dp, syn.seed, args.ttfw_slice_log2, args.ttfw_max_slices,
                                                                dist=dist, device=coll_dev, begin=args.ttfw_begin)

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    cpu = None
    if world == 1 and not args.no_cpu_baseline:   # the CPU baseline is an N=1 figure
        cpu = cpu_baseline(syn, prog, args.cpu_seconds, dev, dp)

    out = {
        "metric": "candidate-assignment evals/sec",
        "value": value,
        "unit": "evals/s",
        "n_gpus": world * max(1, args.devices),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u256 (u32 limbs)",
        "data": "synthetic (Philox-generated candidates, planted witness)",
        "config": {
            "workload": "C5: synthetic 256-bit bitvector DAG, 16 free 256-bit vars, AND of 32 comparisons, "
                        "exhaustive search (BASELINE.json configs[4], per-GPU shard)",
            "dag_nodes": len(__import__("mythril_amd.ir", fromlist=["topo"]).topo(syn.conjuncts)),
            "candidates_per_gpu_step": batch,
            "ops_per_eval": prog.ops_per_eval,
            "ops_per_eval_executed": ops_launch / batch,
            "ops_per_eval_floor": ops_floor / batch,
            "division_paths_per_eval": {k[9:]: v / batch for k, v in per_launch.items()},
            "program_insns": prog.n_insn,
            "spill_slots": prog.n_spill,
            "engine": args.engine + (f" ({dp.kernel}, {args.jit_waves} wave/SIMD, {args.jit_lds_leaves} leaves in LDS, "
                                     f"interleave {args.jit_interleave}, split {jit.SPLIT_KIND})"
                                     if getattr(dp, "kernel", None) else "")
                      + (" [host emulator: CPU test of the rank plumbing, not a measurement]"
                         if args.host_emulator else ""),
            "jit_compile_s": jit_s,
            "jit_split": bool(args.jit_split) if args.engine == "jit" else None,
            "parallelism": f"candidate-shard x{world}" + (f" (one process, {args.devices} devices)"
                                                          if args.devices > 1 else ""),
            "rccl_world": rccl_world,
            "dist_backend": args.dist_backend if dist is not None else None,
            "candidate_begin": args.begin,
            "witness_found_in_timed_range": found_any,
            "timed_launch_flags": "no launch counters (isa.FLAG_NO_COUNT); division paths from an untimed "
                                  "recount of the same launches",
            "evals_timed": timed_evals,
            "evals_counted": sum(st.get("evals", 0) for st in dcounts),
            "time_to_first_witness": ttfw,
        },
        "roofline": {
            "bound": "valu-int32",
            "achieved": achieved / 1e12,
            "peak": THEORETICAL_PEAK / 1e12,
            "unit": "Tops/s (u32)",
            "frac": achieved / THEORETICAL_PEAK,
            # no credit for any division (SURVEY §8(d) ops minus every wide division)
            "frac_floor": (ops_floor / avg_kernel_s) / THEORETICAL_PEAK if avg_kernel_s > 0 else None,
            "valu_issue_frac": valu_issue_frac(prog, batch, getattr(dp, "kernel", None), avg_kernel_s),
            "traffic": load_traffic(prog, batch, getattr(dp, "kernel", None)),
            "kernel_ms_avg": avg_kernel_s * 1e3,
            "peak_source": "MI355X_MICROARCH.md: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz (wave64 VALU op = 2 cycles)",
            "peak_measured": measured_peak / 1e12 if measured_peak else None,
            "frac_measured": achieved / measured_peak if measured_peak else None,
            # (SURVEY §8(d)'s nominal count, every division at all 8 digit steps,
            # is config.ops_per_eval; since the division rewrite most divisions
            # run one step, so a fraction on the nominal count passes 1.0)
            "peak_measured_source": "v_add_u32_e32 with VGPR operands, 8 chains x 8 waves/SIMD "
                                    "(tools/exp/irate.hip; profiles/valu_peak.json)",
        },
        "cpu_baseline": cpu,
    }
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def time_to_first_witness(dev, dp, seed, slice_log2=24, max_slices=128, dist=None, device=None, begin=0):
    """time until the lowest satisfying index in [0, ...) is
    known, searching slices of 2^24 candidates per rank in order with
    stop-after-hit (outside the timed region), at most 2^31 candidates per rank.
    Reported next to the exhaustive rate.  With N ranks, slice k is
    [k N 2^24, (k+1) N 2^24), split into contiguous rank shards, and one
    all-reduce(MIN) per slice ends the search on every rank at the first slice
    holding a witness.  (C5's planted witness sits at index 0x5EED0005 mod 2^31
    = 1 592 590 341 and its conjunct thresholds leave few others, so at N=1
    this times a ~1.6 G-candidate sweep with stop-after-hit.)"""
    from mythril_amd import isa
    from mythril_amd.distributed import shard_range
    flags = isa.FLAG_STOP_AFTER_HIT | isa.FLAG_EARLY_EXIT
    world = dist.get_world_size() if dist is not None else 1
    rank = dist.get_rank() if dist is not None else 0
    span = (1 << slice_log2) * world
    t0 = time.perf_counter()
    for k in range(max_slices):
        b, c = shard_range(begin + k * span, span, rank, world)
        (found,), _ = dev.search([dp], seed, b, c, flags)
        if dist is not None:
            from mythril_amd.distributed import allreduce_min
            (found,) = allreduce_min([found], device=device)
        if found is not None:
            return {"seconds": time.perf_counter() - t0, "index": found, "candidates_searched": (k + 1) * span}
    return {"seconds": time.perf_counter() - t0, "index": None, "candidates_searched": max_slices * span}


def load_measured_peak():
    """The measured v_add_u32 rate (profiles/valu_peak.json), reported beside the
    guide's peak; None when absent."""
    path = os.path.join(ROOT, "profiles", "valu_peak.json")
    try:
        return float(json.load(open(path))["measured_ops_per_s"])
    except Exception:
        return None


def load_pmc(prog, batch, kernel):
    """The committed rocprofv3 PMC record for this kernel and batch
    (profiles/pmc_traffic.json, written by tools/pmc_traffic.py), else None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(path))
    except Exception:
        return None
    # the profile names the launched symbol (<kernel>_x); the attached program
    # carries the module's kernel name
    name = d.get("kernel_name", "?")
    if d.get("ops_per_eval") == prog.ops_per_eval and d.get("batch") == batch and \
            kernel and (name == kernel or name.startswith(kernel + "_")):
        return d
    return None


def load_traffic(prog, batch, kernel):
    """HBM bytes per launch from the committed PMC passes: (2 x FETCH_SIZE +
    WRITE_SIZE) x 1024, the gfx950 correction of MI355X_MICROARCH.md §HBM."""
    d = load_pmc(prog, batch, kernel)
    return d.get("hbm_bytes_per_launch") if d else None


def valu_issue_frac(prog, batch, kernel, kernel_s, n_cu=256, clock_hz=2.4e9):
    """VALU wave-instructions the committed PMC pass counted per launch, over
    what the CUs can issue in the measured kernel time (2 wave64 VALU
    instructions per CU-clock: 4 SIMDs, 2 cycles each), or None."""
    d = load_pmc(prog, batch, kernel)
    if not d or not d.get("sq_insts_valu_per_launch") or kernel_s <= 0:
        return None
    return d["sq_insts_valu_per_launch"] / (kernel_s * n_cu * clock_hz * 2.0)


def cpu_baseline(syn, prog, budget_s, dev, dp):
    """Two CPU legs over bounded samples of the same candidate indices 0..:
    the product's interpreter and ALU built for the host with OpenMP
    (mythril_amd/host_baseline.py; the reported ``value``, SURVEY §8(d)'s
    "build CPU restatement"), and the independent C oracle (oracle/c, bit-serial
    division; ``checker``).  Each leg's verdict vector is compared with the
    GPU's on its indices, and the two legs with each other on their overlap (a
    full-size parity check of the benchmarked kernel)."""
    import numpy as np
    from oracle import cbaseline
    rec, vf = None, None
    from mythril_amd import host_baseline
    if host_baseline.available():
        rec, vf = host_baseline.baseline(prog, syn.seed, budget_s, verdicts=True)
    orc, vo = cbaseline.run(syn, prog, budget_s / 2 if rec else budget_s, verdicts=True)

    def vs_gpu(v):
        vg, _ = dev.eval_generated(dp, syn.seed, 0, len(v), trace=False)
        return int(np.count_nonzero(vg.astype(np.uint8) != v))
    for r, v in ((rec, vf), (orc, vo)):
        if r is not None and v is not None:
            r["verdicts_compared"] = int(len(v))
            r["verdict_mismatches_vs_gpu"] = vs_gpu(v)
            if r["verdict_mismatches_vs_gpu"]:
                print(f"[bench] PARITY FAILURE: {r['verdict_mismatches_vs_gpu']} of {len(v)} CPU verdicts "
                      f"({r['sample'][:40]}...) differ from the GPU's", file=sys.stderr)
    win = witness_window(syn, prog, dev, dp)
    if rec is None:
        orc["witness_window"] = win
        return orc
    if vo is not None:
        k = min(len(vo), len(vf))
        orc["verdict_mismatches_vs_host_build"] = int(np.count_nonzero(vo[:k] != vf[:k]))
    rec["checker"] = orc
    rec["witness_window"] = win
    return rec


def witness_window(syn, prog, dev, dp, half=1 << 12):
    """Mixed-verdict parity at full size (the timed samples above hold no
    satisfying index): the 2*half candidates around the planted witness, each
    verdict from the GPU, the host build and the C oracle, compared."""
    import numpy as np
    from oracle import cdag
    from mythril_amd import host_baseline
    b, n = max(0, syn.witness_index - half), 2 * half
    vg, _ = dev.eval_generated(dp, syn.seed, b, n, trace=False)
    vg = vg.astype(np.uint8)
    out = {"begin": b, "count": n, "satisfied_gpu": int(vg.sum())}
    legs = []
    if host_baseline.available():
        f = host_baseline.specialised(prog)
        _, vh = (host_baseline.count_specialised(f, prog, syn.seed, b, n) if f is not None
                 else host_baseline.count(prog, syn.seed, b, n, verdicts=True))
        legs.append(("host_build", vh))
    if cdag.available():
        _, _, vo = cdag.evaluate(syn.conjuncts, syn.seed, b, n, want_verdict=True)
        legs.append(("oracle", vo))
    for name, v in legs:
        out[f"satisfied_{name}"] = int(v.sum())
        out[f"mismatches_{name}_vs_gpu"] = int(np.count_nonzero(v.astype(np.uint8) != vg))
        if out[f"mismatches_{name}_vs_gpu"]:
            print(f"[bench] PARITY FAILURE: {out[f'mismatches_{name}_vs_gpu']} of {n} verdicts around the "
                  f"planted witness differ ({name} vs GPU)", file=sys.stderr)
    return out

if __name__ == "__main__":
    main()
