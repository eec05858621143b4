#!/bin/bash
# bounding-kernel parity (all formats, sieve, scale), then C4 / C5 with PACKED64 vs PACKED_WIDE (TAG = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4f}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_sieve.py tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
bash tools/gpu_matrix.sh ${1:-r4f}/m tools/m_c45b.txt
