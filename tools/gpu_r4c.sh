#!/bin/bash
# phase clock of C3 (abv_keep/phase.so), then the abv variants interleaved (TAG = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4c}
mkdir -p $OUT
PIPELINEDP_AMD_LIB=$PWD/abv_keep/phase.so timeout -k 10 240 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --no-api > $OUT/phase_c3.log 2>&1 || { tail -5 $OUT/phase_c3.log; exit 1; }
grep -E "^l1 |^phase" $OUT/phase_c3.log | head -24
BENCH_ARGS="--no-api --no-secondary" bash tools/gpu_variants.sh ${1:-r4c}/v
