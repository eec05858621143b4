#!/bin/bash
# Round 4: the whole -m gpu suite, the C3/C4/C5 bench lines, then phase-clock
# runs of C4 and C5 (abv/phase.so); stops at the first failure (TAG = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4b}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
cat > $OUT/m.txt <<'M'
c3|--steps 10 --warmup 3 --no-api
c4|--workload c4 --steps 5 --warmup 2
c5|--workload c5 --steps 5 --warmup 2
M
bash tools/gpu_matrix.sh ${1:-r4b}/m $OUT/m.txt || exit 1
bash tools/gpu_phase.sh ${1:-r4b}/ph4 --workload c4 || exit 1
bash tools/gpu_phase.sh ${1:-r4b}/ph5 --workload c5 || exit 1
echo "r4b ok"
