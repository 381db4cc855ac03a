set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
echo "== opbench jit"
timeout -k 10 300 python3 tools/opbench.py jit 2>&1 | tail -20 || exit 1
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline"
i=0
for set in "SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA" \
           "SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_INSTS_LDS,SQ_INSTS_BRANCH,SQ_INSTS_VMEM,SQ_INST_CYCLES_SALU,SQ_INSTS_FLAT" \
           "FETCH_SIZE" "WRITE_SIZE" ; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc/p$i -o run -- $B > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
done
find gpurun_out/pmc -name "*counter_collection*"
