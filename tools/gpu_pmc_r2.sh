#!/bin/bash
# HBM bytes per kernel for the bench workloads (round 2): separate rocprofv3
# --pmc passes for FETCH_SIZE and WRITE_SIZE (MI355X_MICROARCH.md: one TCC
# group per pass), each over `bench.py --workload W` alone, then
# tools/pmc_summary.py -> profiles/r02/W_pmc.json with the tag bench.py
# checks ("W n=<rows per GPU> ").  Every pass has its own time limit and the
# script stops at the first failure.
# Usage: bash tools/gpu_pmc_r2.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-pmc_r2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
declare -A ROWS=([c3]=1000000000 [c2]=100000000)
for W in c3 c2; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $C -d $OUT/$W/$C -o run --output-format csv -- python -u bench.py --workload $W --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --no-api > $OUT/${W}_$C.log 2>&1 || { echo "PMC pass $W $C failed"; tail -5 $OUT/${W}_$C.log; exit 1; }
  done
  python3 tools/pmc_summary.py $OUT/$W $OUT/${W}_pmc.json "$W n=${ROWS[$W]} tree=$(cat .tree_id 2>/dev/null || echo unknown)" || exit 1
done
echo "pmc ok"
