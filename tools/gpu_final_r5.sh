#!/bin/bash
# Round-5 tree: the whole GPU suite, smoke(), then the bench lines (TAG = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-fin5}
OUT=gpurun_out/$T
mkdir -p $OUT
rocm-smi --showmeminfo vram > $OUT/smi.txt 2>&1 || true
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "BENCH FAILED"; tail -20 $OUT/bench.err; exit 1; }
for a in "c4|--workload c4 --steps 5 --warmup 2" "c4g|--workload c4 --steps 5 --warmup 2 --strategy gaussian" "c5|--workload c5 --steps 5 --warmup 2" "hist|--workload hist" "c3small|--small-ids 0.3 --steps 10 --warmup 3 --no-secondary --no-api --no-cpu-baseline" "c3share8|--share-of 8 --steps 20 --warmup 5 --no-api --no-cpu-baseline"; do
  n=${a%%|*}; x=${a#*|}
  timeout -k 10 400 python -u bench.py $x > $OUT/bench_$n.json 2> $OUT/bench_$n.err || { echo "BENCH $n FAILED"; tail -20 $OUT/bench_$n.err; exit 1; }
  echo "$n ok"
done
python3 tools/bench_summary.py $OUT/bench.json $OUT/bench_c4.json $OUT/bench_c4g.json $OUT/bench_c5.json $OUT/bench_hist.json $OUT/bench_c3small.json $OUT/bench_c3share8.json
fi
