set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
grep -oE "SQ_[A-Z_0-9]+" gpurun_out/pmc/counters.txt | sort -u > gpurun_out/pmc/sq_counters.txt || true
wc -l gpurun_out/pmc/sq_counters.txt
i=0
for set in "SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA" \
           "SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_INSTS_LDS,SQ_INSTS_BRANCH,SQ_WAIT_INST_LDS,SQ_INSTS_VMEM,SQ_INST_CYCLES_SALU" ; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 tools/pmc_probe.py bvxor > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; }
done
find gpurun_out/pmc -name "*counter_collection*" | head
