set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pools4
echo "== gpu tests"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pools4/gpu_tests.log 2>&1; rc=$?; tail -4 gpurun_out/pools4/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== replay"
timeout -k 10 300 python3 -m mythril_amd.replay tests/golden/solver_log > gpurun_out/pools4/replay.txt 2>&1 || { tail gpurun_out/pools4/replay.txt; exit 1; }
cat gpurun_out/pools4/replay.txt
echo "== C2-C4 config bench"
timeout -k 10 400 python3 tools/config_bench.py --out gpurun_out/pools4/config_bench.json > gpurun_out/pools4/config_bench.log 2>&1 || { tail gpurun_out/pools4/config_bench.log; exit 1; }
cat gpurun_out/pools4/config_bench.log
