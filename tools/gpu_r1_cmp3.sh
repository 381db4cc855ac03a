set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== gpu tests"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for sp in 1 0; do
echo "== bench jit split=$sp"
timeout -k 10 600 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --jit-split $sp > gpurun_out/bench_s$sp.json 2> gpurun_out/bench_s$sp.err || { tail -5 gpurun_out/bench_s$sp.err; exit 1; }
cat gpurun_out/bench_s$sp.json
done
echo "== opbench jit"
timeout -k 10 300 python3 tools/opbench.py jit 2>&1 | tail -16 || exit 1
