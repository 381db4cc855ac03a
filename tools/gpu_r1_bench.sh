set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "== smoke"
timeout -k 10 240 python3 -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -3 || exit 1
echo "== gpu tests"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"
timeout -k 10 600 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -5 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
echo "== rocprof kernel trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/bench_prof.json 2>gpurun_out/bench_prof.err || { tail -5 gpurun_out/bench_prof.err; exit 1; }
cat gpurun_out/bench_prof.json
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline"
mkdir -p gpurun_out/pmc
i=0
for set in "SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA" \
           "SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_INSTS_LDS,SQ_INSTS_BRANCH,SQ_INSTS_VMEM,SQ_INST_CYCLES_SALU,SQ_INSTS_FLAT" \
           "FETCH_SIZE" "WRITE_SIZE" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc/p$i -o run -- $B > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
done
echo pmc done
echo "== torchrun (1 rank, RCCL path)"
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 1 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_torchrun.json 2> gpurun_out/bench_torchrun.err || { tail -5 gpurun_out/bench_torchrun.err; exit 1; }
cat gpurun_out/bench_torchrun.json
