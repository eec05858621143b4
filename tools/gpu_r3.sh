#!/bin/bash
# Round-3 GPU step: parity tests, the default bench line, then the A/B
# variants in abv/ (tools/build_variants.sh); stops at the first failure.
# Usage: bash tools/gpu_r3.sh TAG [skip-tests]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-api > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
python3 tools/bench_summary.py $OUT/bench.json 2>/dev/null || tail -c 600 $OUT/bench.json
timeout -k 10 300 python -u bench.py --workload hist --steps 5 --warmup 2 > $OUT/bench_hist.json 2> $OUT/bench_hist.err || { echo "HIST BENCH FAILED"; tail -20 $OUT/bench_hist.err; exit 1; }
python3 tools/bench_summary.py $OUT/bench_hist.json 2>/dev/null || tail -c 600 $OUT/bench_hist.json
if ls abv/*.so > /dev/null 2>&1; then bash tools/gpu_variants.sh $TAG/v || exit 1; fi
echo "r3 step ok"
