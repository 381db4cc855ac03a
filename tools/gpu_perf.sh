set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 tools/opbench.py 2>&1 | tail -20 || exit 1
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline 2>&1 | tail -3
