#!/bin/bash
# One GPU lease: [pytest selection] [smoke] [bench lines].  Results under gpurun_out/$TAG.
#   TAG=r6a TESTS="tests/test_gpu_sieve.py tests/test_gpu_api.py" SMOKE=1 \
#   BENCH="main|--steps 20 --warmup 5;share8|--share-of 8 --no-api --no-cpu-baseline" tools/gpu_run.sh
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-1000} python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread \
    > "$OUT/pytest_gpu.log" 2>&1 || { echo "PYTEST FAILED"; tail -40 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
fi
if [ "${SMOKE:-0}" = 1 ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
    || { echo "SMOKE FAILED"; tail -20 "$OUT/smoke.log"; exit 1; }
  tail -2 "$OUT/smoke.log"
fi
IFS=';' read -ra LINES <<< "$BENCH"
for a in "${LINES[@]}"; do
  [ -z "$a" ] && continue
  n=${a%%|*}; x=${a#*|}
  timeout -k 10 ${BENCH_TIMEOUT:-400} python -u bench.py $x > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" \
    || { echo "BENCH $n FAILED"; tail -20 "$OUT/bench_$n.err"; exit 1; }
  echo "$n ok"
done
if [ -n "$BENCH" ]; then python3 tools/bench_summary.py "$OUT"/bench_*.json; fi
