#!/bin/bash
# One parameterised GPU-box recipe (run under gpurun):
#
#   tools/gpu_run.sh TAG STEP [STEP...]
#
# Steps (each under its own time limit; the script stops at the first failure):
#   smoke          __graft_entry__.smoke()
#   tests[=EXPR]   pytest -m gpu (optionally -k EXPR)
#   quick=EXPR     pytest -m gpu -k EXPR under a 180 s limit (first runs of new kernels)
#   bench          python bench.py (default flags) -> bench.json
#   bench1         bench.py --steps 5 --no-ttfw --no-cpu-baseline $BENCH_ARGS (quick A/B runs)
#   prof           rocprofv3 --kernel-trace --stats on a short bench run
#   pmc            PMC passes on one bench launch (SQ, instruction mix, FETCH_SIZE, WRITE_SIZE)
#   config         tools/config_bench.py (C2-C4 queries) -> config_bench.json
#   gt[=LOG2]      tools/ground_truth.py: the corpus's unknown queries searched up to 2^LOG2 (32)
#   latency        tools/latency_bench.py (drop-in prepare/search/materialise per query)
#   dropinprof     tools/dropin_profile.py (library step times per drop-in query)
#   replay         python -m mythril_amd.replay tests/golden/solver_log
#   replaylat      tools/replay_latency.py (LASER-order translation + preparation, host only)
#   c3prep         tools/c3_prepare.py (C3 through the per-conjunct cache, host only)
#   opbench        tools/opbench.py jit
#   keccak         tools/keccak_bench.py
#   ipmc=FILE      PMC passes on one exhaustive interpreter launch of FILE (tools/interp_once.py)
#   jpmc=FILE      the same on FILE's cached specialised kernel
#   apmc=FILE      the same on FILE's assembled kernel (mythril_amd/asmjit.py)
#   opcost         tools/interp_opcost.py (+ one PMC pass: instructions per bytecode op)
#   ablate         tools/leaf_ablate.py --run (candidate-generation ablations, C2/C2L/C4)
#   recip          tools/exp/recip_check (device reciprocal vs u64 division; built by hand)
#   ab=V1,V2       tools/ab_c5.py: C5 code-generation variants (compiled beforehand), timed and cross-checked
# Outputs land in gpurun_out/TAG/.
set -o pipefail
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-ttfw --no-recount ${BENCH_ARGS:-}"

run() {  # run LIMIT LOG CMD...: one GPU step, bounded; print the log tail on failure
  local lim=$1 log=$2
  shift 2
  timeout -k 10 "$lim" "$@" > "$log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "step failed rc=$rc: $*"
    tail -30 "$log"
    exit $rc
  fi
}

for step in "$@"; do
  echo "== $step ($(date +%T))"
  case $step in
    smoke)
      run 240 "$OUT/smoke.log" python3 -c "import __graft_entry__ as g; g.smoke()"
      tail -2 "$OUT/smoke.log" ;;
    quick=*)
      run 180 "$OUT/gpu_quick.log" python3 -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread -k "${step#quick=}"
      tail -3 "$OUT/gpu_quick.log" ;;
    tests|tests=*)
      K=()
      [ "$step" != tests ] && K=(-k "${step#tests=}")
      run 1000 "$OUT/gpu_tests.log" python3 -u -m pytest tests -m gpu -x -v -s --timeout 150 --timeout-method thread "${K[@]}"
      tail -3 "$OUT/gpu_tests.log" ;;
    bench)
      run 500 "$OUT/bench.err" bash -c "python3 bench.py > $OUT/bench.json"
      cat "$OUT/bench.json" ;;
    bench1)
      run 300 "$OUT/bench1.err" bash -c "${B/--no-recount/} > $OUT/bench1.json"
      cat "$OUT/bench1.json" ;;
    prof)
      run 400 "$OUT/prof.log" rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- $B
      find "$OUT/prof" -name "*kernel_stats.csv" -exec head -5 {} \; ;;
    pmc)
      i=0
      for set in "SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA" \
                 "SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_INSTS_LDS,SQ_INSTS_BRANCH,SQ_INSTS_VMEM,SQ_INST_CYCLES_SALU,SQ_INSTS_FLAT" \
                 "FETCH_SIZE" "WRITE_SIZE"; do
        i=$((i + 1))
        run 150 "$OUT/pmc$i.log" timeout -s KILL 140 rocprofv3 --pmc $set --output-format csv -d "$OUT/pmc/p$i" -o run -- \
          python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ttfw --no-recount
      done
      find "$OUT/pmc" -name "*counter_collection*" ;;
    config)
      run 600 "$OUT/config_bench.log" python3 tools/config_bench.py --out "$OUT/config_bench.json"
      tail -12 "$OUT/config_bench.log" ;;
    gt|gt=*)
      G=()
      [ "$step" != gt ] && G=(--max-log2 "${step#gt=}")
      run 1100 "$OUT/ground_truth.log" python3 -u tools/ground_truth.py --out "$OUT/ground_truth.json" "${G[@]}"
      tail -8 "$OUT/ground_truth.log" ;;
    latency)
      run 600 "$OUT/latency.log" python3 tools/latency_bench.py --out "$OUT/latency.json"
      tail -20 "$OUT/latency.log" ;;
    dropinprof)
      run 300 "$OUT/dropin_profile.log" python3 tools/dropin_profile.py --out "$OUT/dropin_profile.json"
      head -60 "$OUT/dropin_profile.log" ;;
    dropinab)   # the same under each A/B environment (tools/dropin_profile.py --ab)
      run 900 "$OUT/dropin_ab.log" python3 tools/dropin_profile.py --ab --out "$OUT/dropin_ab.json"
      tail -30 "$OUT/dropin_ab.log" ;;
    replay)
      run 300 "$OUT/replay.txt" python3 -m mythril_amd.replay tests/golden/solver_log
      tail -12 "$OUT/replay.txt" ;;
    c3prep)
      run 300 "$OUT/c3_prepare.log" python3 -u tools/c3_prepare.py --reps 40 --out "$OUT/c3_prepare.json"
      tail -2 "$OUT/c3_prepare.log" ;;
    replaylat)
      run 400 "$OUT/replay_latency.log" python3 -u tools/replay_latency.py --out "$OUT/replay_latency.json"
      tail -3 "$OUT/replay_latency.log" ;;
    opbench)
      run 400 "$OUT/opbench.log" python3 tools/opbench.py jit
      tail -20 "$OUT/opbench.log" ;;
    keccak)
      run 300 "$OUT/keccak.log" python3 tools/keccak_bench.py
      tail -8 "$OUT/keccak.log" ;;
    ab=*)
      run 300 "$OUT/ab_c5.log" python3 -u tools/ab_c5.py --variants "${step#ab=}" --out "$OUT/ab_c5.json" || exit 1
      cat "$OUT/ab_c5.log" ;;
    ipmc=*|jpmc=*|apmc=*)
      F=${step#*=}
      J=()
      P=${step%%=*}
      [ "$P" = jpmc ] && J=(--jit)
      [ "$P" = apmc ] && J=(--asmjit)
      i=0
      for set in "SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA" \
                 "SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_INSTS_LDS,SQ_INSTS_BRANCH,SQ_INSTS_VMEM,SQ_INST_CYCLES_SALU,SQ_INSTS_FLAT" \
                 "SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_LDS,SQ_ACTIVE_INST_VMEM,SQ_LDS_BANK_CONFLICT"; do
        i=$((i + 1))
        run 150 "$OUT/$P$i.log" timeout -s KILL 140 rocprofv3 --pmc $set --output-format csv -d "$OUT/$P/p$i" -o run -- \
          python3 tools/interp_once.py "$F" 22 "${J[@]}"
      done
      find "$OUT/$P" -name "*counter_collection*" ;;
    opcost)
      run 300 "$OUT/opcost.log" python3 tools/interp_opcost.py
      cat "$OUT/opcost.log"
      run 200 "$OUT/opcost_pmc.log" timeout -s KILL 190 rocprofv3 --pmc SQ_WAVES,SQ_WAVE_CYCLES,SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_INSTS_BRANCH,SQ_WAIT_INST_ANY,SQ_WAIT_ANY \
        --output-format csv -d "$OUT/opcost_pmc" -o run -- python3 tools/interp_opcost.py --log2 18
      find "$OUT/opcost_pmc" -name "*counter_collection*" ;;
    ablate)
      run 1200 "$OUT/ablate.log" python3 tools/leaf_ablate.py --run "$OUT/ablate"
      tail -30 "$OUT/ablate.log" ;;
    asmdiff)
      run 300 "$OUT/asm_diff.log" python3 tools/asm_diff.py
      tail -20 "$OUT/asm_diff.log" ;;
    recip)
      run 120 "$OUT/recip.txt" ./tools/exp/recip_check
      tail -4 "$OUT/recip.txt" ;;
    *)
      echo "unknown step $step"
      exit 2 ;;
  esac
done
echo "== done ($(date +%T))"
