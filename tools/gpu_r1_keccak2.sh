set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/keccak2
echo "== keccak parity"
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "keccak or smoke or native" > gpurun_out/keccak2/tests.log 2>&1; rc=$?; tail -3 gpurun_out/keccak2/tests.log; [ $rc -eq 0 ] || exit $rc
echo "== keccak bench under rocprof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/keccak2/prof -o run --output-format csv -- python3 tools/keccak_bench.py > gpurun_out/keccak2/bench.log 2>&1 || { tail gpurun_out/keccak2/bench.log; exit 1; }
tail -5 gpurun_out/keccak2/bench.log
cp gpurun_out/keccak_bench.json gpurun_out/keccak2/ 2>/dev/null
cut -d, -f1-4 gpurun_out/keccak2/prof/run_kernel_stats.csv | head -4
