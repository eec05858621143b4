#!/bin/bash
# round 5: counters available on the box, then ROUNDS interleaved bench passes over abv/*.so (TAG = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r5b}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/avail.txt 2>&1 || echo "list-avail rc=$?"
ROUNDS=${ROUNDS:-3} BENCH_ARGS="--no-api --no-secondary" bash tools/gpu_variants.sh $T/c3
