#!/bin/bash
# round 5: u16 bucket counts -- parity, then A/B on C3, share-of-8, C4, C5 (TAG = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r5p}
OUT=gpurun_out/$T
mkdir -p $OUT
PIPELINEDP_AMD_LIB=$PWD/abv/u16.so timeout -k 10 600 python -u -m pytest tests/test_gpu_sieve.py tests/test_gpu_scale.py tests/test_gpu_kernels.py -x -q --timeout 250 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -30 $OUT/pytest.log; exit 1; }
echo "parity u16: $(tail -1 $OUT/pytest.log)"
ROUNDS=2 BENCH_ARGS="--no-api --no-secondary" bash tools/gpu_variants.sh $T/c3 && \
ROUNDS=1 BENCH_ARGS="--no-api --share-of 8 --steps 20" bash tools/gpu_variants.sh $T/share8 && \
ROUNDS=1 BENCH_ARGS="--no-api --workload c4" bash tools/gpu_variants.sh $T/c4 && \
ROUNDS=1 BENCH_ARGS="--no-api --workload c5 --steps 5 --warmup 2" bash tools/gpu_variants.sh $T/c5
