#!/bin/bash
# sieve parity with the 512-thread fix-up launches, then A/B: C3 two rounds, the light-user variant one (TAG = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r4m}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_sieve.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
ROUNDS=2 BENCH_ARGS="--no-secondary --no-api" bash tools/gpu_variants.sh $T/c3 && ROUNDS=1 BENCH_ARGS="--small-ids 0.3 --steps 5 --warmup 2 --no-secondary --no-api" bash tools/gpu_variants.sh $T/small
