set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== probe"; python3 -c "import z3" 2>&1 | tail -1; which solc || echo "no solc"
echo "== smoke"
timeout -k 10 240 python3 -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -3 || exit 1
echo "== gpu tests"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -5 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --cpu-seconds 10 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -5 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
echo "== rocprof kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof.json 2>gpurun_out/bench_prof.err || { tail -5 gpurun_out/bench_prof.err; exit 1; }
cat gpurun_out/bench_prof.json
find gpurun_out/prof -name "*stats*"
