#!/bin/bash
# A/B of two builds of the product library on the asm interpreter (config
# bench C2-C4 + LASER group, twice each way, alternating):
#   bash tools/ab_lib.sh TAG OTHER.so      (under gpurun; OTHER.so is "A", the in-tree build "B")
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/$1
OTHER=$2
mkdir -p "$OUT"
for r in 1 2; do
  for m in A B; do
    if [ $m = A ]; then export MYTHRIL_AMD_LIB=$PWD/$OTHER; else unset MYTHRIL_AMD_LIB; fi
    timeout -k 10 300 python3 tools/config_bench.py --engines asm --out "$OUT/lib${m}_$r.json" > "$OUT/lib${m}_$r.log" 2>&1 \
      || { tail -20 "$OUT/lib${m}_$r.log"; exit 1; }
    python3 -c "
import json,sys
for l in json.load(open('$OUT/lib${m}_$r.json')): print('$m round $r:', l['config'], round(l['evals_per_s']/1e9, 3), 'G')"
  done
done
