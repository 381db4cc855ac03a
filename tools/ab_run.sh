#!/bin/bash
# A/B interpreter builds on the GPU box: config_bench (interpreter only) with
# the in-tree library (A) and, if present, build/ab/libB.so (B).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/ab
ONLY=${ONLY:-C2,C3,C4,C2L}
timeout -k 10 300 python3 tools/config_bench.py --no-jit --only "$ONLY" --out gpurun_out/ab/A.json > gpurun_out/ab/A.log 2>&1 || exit $?
if [ -f build/ab/libB.so ]; then
  MYTHRIL_AMD_LIB=$PWD/build/ab/libB.so timeout -k 10 300 python3 tools/config_bench.py --no-jit --only "$ONLY" \
    --out gpurun_out/ab/B.json > gpurun_out/ab/B.log 2>&1 || exit $?
fi
