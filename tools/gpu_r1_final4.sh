set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final4
echo "== smoke"
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -3 || exit 1
echo "== gpu tests"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final4/gpu_tests.log 2>&1; rc=$?; tail -4 gpurun_out/final4/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== bench (default)"
timeout -k 10 400 python3 bench.py > gpurun_out/final4/bench.json 2> gpurun_out/final4/bench.err || { tail -5 gpurun_out/final4/bench.err; exit 1; }
cat gpurun_out/final4/bench.json
echo "== rocprof kernel trace + stats"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/final4/prof -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-ttfw > gpurun_out/final4/bench_prof.json 2>gpurun_out/final4/bench_prof.err || { tail gpurun_out/final4/bench_prof.err; exit 1; }
cat gpurun_out/final4/bench_prof.json
echo "== replay"
timeout -k 10 300 python3 -m mythril_amd.replay tests/golden/solver_log > gpurun_out/final4/replay.txt 2>&1 || { tail gpurun_out/final4/replay.txt; exit 1; }
tail -20 gpurun_out/final4/replay.txt
echo "== C2-C4 config bench"
timeout -k 10 400 python3 tools/config_bench.py --out gpurun_out/final4/config_bench.json > gpurun_out/final4/config_bench.log 2>&1 || { tail gpurun_out/final4/config_bench.log; exit 1; }
cat gpurun_out/final4/config_bench.log
