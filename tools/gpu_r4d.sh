#!/bin/bash
# the whole -m gpu suite, then the abv variants interleaved (TAG = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4d}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
BENCH_ARGS="--no-api --no-secondary" bash tools/gpu_variants.sh ${1:-r4d}/v
