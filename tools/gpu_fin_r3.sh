#!/bin/bash
# Round-3 final GPU step: the whole -m gpu suite, then the bench lines the
# driver and DESIGN.md quote (C3 default with its CPU baselines and the C2
# secondary, hist, C4 with truncated-geometric and Gaussian selection, C5),
# each under its own time limit; stops at the first failure.
# Usage: bash tools/gpu_fin_r3.sh TAG [skip-tests]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-fin_r3}
mkdir -p $OUT
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload hist --steps 10 --warmup 3 > $OUT/bench_hist.json 2> $OUT/bench_hist.err || { echo "HIST BENCH FAILED"; tail -20 $OUT/bench_hist.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { echo "C4 BENCH FAILED"; tail -20 $OUT/bench_c4.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload c4 --strategy gaussian --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_c4_gauss.json 2> $OUT/bench_c4_gauss.err || { echo "C4 GAUSS BENCH FAILED"; tail -20 $OUT/bench_c4_gauss.err; exit 1; }
timeout -k 10 400 python -u bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { echo "C5 BENCH FAILED"; tail -20 $OUT/bench_c5.err; exit 1; }
echo "fin ok"
