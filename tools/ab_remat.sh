#!/bin/bash
# A/B of the allocators' leaf rematerialisation (MYTHRIL_AMD_REMAT_LEAVES) on
# the asm interpreter: config bench (C2-C4, LASER group) twice each way,
# alternating.  Run under gpurun: bash tools/ab_remat.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
OUT=gpurun_out/$1
mkdir -p "$OUT"
for r in 1 2; do
  for m in 0 1; do
    MYTHRIL_AMD_REMAT_LEAVES=$m timeout -k 10 300 python3 tools/config_bench.py --engines asm \
      --out "$OUT/remat${m}_$r.json" > "$OUT/remat${m}_$r.log" 2>&1 || { tail -20 "$OUT/remat${m}_$r.log"; exit 1; }
    grep -o '"config": "[A-Z0-9]*".*"evals_per_s": [0-9.e+]*' "$OUT/remat${m}_$r.log" | sed -e 's/"files.*"evals_per_s"/ evals_per_s/' | sed "s/^/remat=$m round $r: /"
  done
done
