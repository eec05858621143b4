#!/bin/bash
# Phase-clock build (abv/phase.so, -DPDP_PHASE_CLOCK): per-tile level-1 / level-2 /
# bucket-kernel phase times printed by sampled workgroups (TAG = $1; extra bench args after)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-phase}
shift
mkdir -p $OUT
PIPELINEDP_AMD_LIB=$PWD/abv/phase.so timeout -k 10 240 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --no-api "$@" > $OUT/phase.log 2>&1 || { tail -5 $OUT/phase.log; exit 1; }
grep -E "^l1 |^l2 |^phase" $OUT/phase.log | head -40
