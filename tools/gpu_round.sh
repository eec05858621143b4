#!/bin/bash
# Full GPU pass for one tag: GPU tests, bench (with CPU baseline), rocprofv3
# kernel stats, PMC HBM-byte passes.  Every GPU step has its own time limit and
# the script stops at the first failure.  Usage: bash tools/gpu_round.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-round}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; echo "PYTEST FAILED"; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; echo "BENCH FAILED"; exit 1; }
tail -1 $OUT/bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; echo "ROCPROF FAILED"; exit 1; }
for C in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  N=$(echo $C | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmc/$N -o run --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmc_$N.log 2>&1 || { echo "PMC pass $C failed"; exit 1; }
done
python3 tools/pmc_summary.py $OUT/pmc $OUT/pmc.json "C2 bench.py --steps 3 --warmup 1"
