#!/bin/bash
# A/B of the abv/ variants: C3 (+C2) two rounds, C4 and C5 one round (TAG = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-r4l}
ROUNDS=2 bash tools/gpu_variants.sh $T/c3 && ROUNDS=1 BENCH_ARGS="--workload c4 --steps 5 --warmup 2" bash tools/gpu_variants.sh $T/c4 && ROUNDS=1 BENCH_ARGS="--workload c5 --steps 5 --warmup 2" bash tools/gpu_variants.sh $T/c5
