set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
echo "== opbench"
timeout -k 10 300 python3 tools/opbench.py 2>&1 | tail -30 || exit 1
echo "== rocprof kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_prof.json 2>gpurun_out/bench_prof.err || { tail gpurun_out/bench_prof.err; exit 1; }
cat gpurun_out/bench_prof.json
find gpurun_out/prof_r1 -name "*stats*" | head
