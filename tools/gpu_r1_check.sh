set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== gpu tests"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"
timeout -k 10 600 python3 bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -5 gpurun_out/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench.json')); print(d['value']/1e6, 'M evals/s', d['roofline']['frac'], d['config']['time_to_first_witness'])"
echo "== opbench jit"
timeout -k 10 300 python3 tools/opbench.py jit 2>&1 | tail -3 || exit 1
