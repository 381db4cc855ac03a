set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
echo "== probe"; python3 -c "import z3" 2>&1 | tail -1; python3 -c "import mythril" 2>&1 | tail -1; which solc || echo "no solc"
echo "== smoke"
timeout -k 10 180 python3 -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -5 || exit 1
echo "== gpu tests"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r1.log 2>&1; rc=$?; tail -25 gpurun_out/gpu_tests_r1.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --cpu-seconds 5 > gpurun_out/bench_r1.json 2> gpurun_out/bench_r1.err; rc=$?; cat gpurun_out/bench_r1.json; tail -5 gpurun_out/bench_r1.err; exit $rc
