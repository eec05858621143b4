#!/bin/bash
# half-size bucket workgroups: parity, then the bench matrix tools/m_bt.txt (TAG = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r4i}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_sieve.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/gpu_matrix.sh $T/m tools/m_bt.txt
