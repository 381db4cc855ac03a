set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
ls build/jit | head
echo "== gpu tests"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -5 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== bench jit"
timeout -k 10 600 python3 bench.py --steps 3 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_jit.json 2> gpurun_out/bench_jit.err || { tail -5 gpurun_out/bench_jit.err; exit 1; }
cat gpurun_out/bench_jit.json
echo "== rocprof kernel trace (jit)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_jit -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_jit_prof.json 2>gpurun_out/bench_jit_prof.err || { tail -5 gpurun_out/bench_jit_prof.err; exit 1; }
cat gpurun_out/bench_jit_prof.json
