#!/bin/bash
# Round-2 GPU pass for one tag: GPU tests, default bench (C3 + C2 secondary +
# CPU baselines), rocprofv3 kernel stats of the C3 bench.  Every GPU step has
# its own time limit and the script stops at the first failure.
# Usage: bash tools/gpu_r2.sh TAG [pytest args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r2}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
TESTS=${@:-tests}
timeout -k 10 1100 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; echo "PYTEST FAILED"; exit 1; }
tail -3 $OUT/pytest_gpu.log
if [ -n "${NO_BENCH:-}" ]; then exit 0; fi
timeout -k 10 400 python -u bench.py > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; echo "BENCH FAILED"; exit 1; }
python3 tools/bench_summary.py $OUT/bench.log
if [ -n "${NO_PROF:-}" ]; then exit 0; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; echo "ROCPROF FAILED"; exit 1; }
echo "rocprof ok"
