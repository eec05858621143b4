#!/bin/bash
# round 5: level-1 placement A/B. Parity of the padded + contiguous variant on
# the sieve tests, then ROUNDS interleaved bench passes over abv/*.so (TAG = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r5a}
OUT=gpurun_out/$T
mkdir -p $OUT
PIPELINEDP_AMD_LIB=$PWD/abv/both.so timeout -k 10 400 python -u -m pytest tests/test_gpu_sieve.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
ROUNDS=${ROUNDS:-4} BENCH_ARGS="--no-api" bash tools/gpu_variants.sh $T/c3
