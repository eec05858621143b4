#!/bin/bash
# selection / noise parity, then C4 with Gaussian thresholding and truncated geometric (TAG = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r4h}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_thresholding.py tests/test_gpu_api.py tests/test_gpu_kernels.py tests/test_secure_noise.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/gpu_matrix.sh $T/m tools/m_c4g.txt
