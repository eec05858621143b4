#!/bin/bash
# GPU pass for the dataset histograms: parity tests, bench, rocprofv3 kernel
# stats.  Every GPU step has its own time limit; stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-hist}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_histograms.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_hist.log 2>&1 || { tail -40 $OUT/pytest_hist.log; echo "PYTEST FAILED"; exit 1; }
tail -3 $OUT/pytest_hist.log
timeout -k 10 300 python -u tools/bench_hist.py > $OUT/bench_hist.log 2>&1 || { tail -20 $OUT/bench_hist.log; echo "BENCH FAILED"; exit 1; }
tail -1 $OUT/bench_hist.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python -u tools/bench_hist.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; echo "ROCPROF FAILED"; exit 1; }
echo PROF OK
