#!/bin/bash
# A/B + PMC of the C5 kernel variants in the in-tree cache (tools/ab_c5.py)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1
V=${2:-asm}
mkdir -p $OUT
timeout -k 10 200 python3 tools/ab_c5.py --variants $V --out $OUT/ab.json > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
tail -3 $OUT/ab.log
i=0
for set in "SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA" \
           "SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_SMEM,SQ_INSTS_LDS,SQ_INSTS_BRANCH,SQ_INSTS_VMEM,SQ_INST_CYCLES_SALU,SQ_INSTS_FLAT"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc/p$i -o run -- python3 tools/ab_c5.py --variants $V --reps 1 --out $OUT/abp$i.json > $OUT/pmc$i.log 2>&1 || { tail -20 $OUT/pmc$i.log; exit 1; }
done
find $OUT/pmc -name "*counter_collection*"
