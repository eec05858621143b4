#!/bin/bash
# GPU round trip: parity tests -> bench -> rocprofv3 kernel trace (TAG = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-check}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -15 $OUT/pytest.log
if [ $rc -ne 0 ]; then echo "PYTEST FAILED rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 ${BENCH_ARGS:-} > $OUT/bench.log 2>&1
rc=$?
tail -2 $OUT/bench.log
if [ $rc -ne 0 ]; then echo "BENCH FAILED rc=$rc"; exit $rc; fi
if [ -z "${NO_PROF:-}" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1
  rc=$?
  find $OUT/prof -name "*kernel_stats.csv" -exec cat {} \; | head -30
  exit $rc
fi
