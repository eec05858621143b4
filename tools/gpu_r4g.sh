#!/bin/bash
# bounding-kernel parity, then range-major run table A/B: C3 (+C2) and C5 (TAG = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r4g}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_sieve.py tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
ROUNDS=2 bash tools/gpu_variants.sh $T/c3 && ROUNDS=1 BENCH_ARGS="--workload c5 --steps 5 --warmup 2" bash tools/gpu_variants.sh $T/c5
