#!/bin/bash
# A/B of abv/*.so on C3 and on one rank's share of an 8-GPU C3 run, with
# optional parity first ($PARITY variant, $PARITY_TESTS), TAG = $1
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-abx}
OUT=gpurun_out/$T
mkdir -p $OUT
rocm-smi --showmeminfo vram > $OUT/smi.txt 2>&1 || true
if [ -n "$PARITY_TESTS" ]; then
  PIPELINEDP_AMD_LIB=$PWD/abv/$PARITY.so timeout -k 10 500 python -u -m pytest $PARITY_TESTS -x -q --timeout 250 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -30 $OUT/pytest.log; exit 1; }
  echo "parity $PARITY: $(tail -1 $OUT/pytest.log)"
fi
ROUNDS=${ROUNDS:-2} BENCH_ARGS="--no-api --no-secondary $C3_ARGS" bash tools/gpu_variants.sh $T/c3 && \
ROUNDS=${ROUNDS:-2} BENCH_ARGS="--no-api --share-of 8 --steps 20" bash tools/gpu_variants.sh $T/share8
