#!/bin/bash
# Dataset histograms: GPU parity tests, then PMC HBM-byte passes (one counter
# group per run) over a short tools/bench_hist.py run.  Usage: bash tools/gpu_hist_pmc.sh TAG
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-hist_pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_histograms.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_hist.log 2>&1 || { tail -40 $OUT/pytest_hist.log; echo "PYTEST FAILED"; exit 1; }
tail -3 $OUT/pytest_hist.log
for C in "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/pmc/$C -o run --output-format csv -- python -u tools/bench_hist.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/pmc_$C.log 2>&1 || { tail -20 $OUT/pmc_$C.log; echo "PMC pass $C failed"; exit 1; }
done
python3 tools/pmc_summary.py $OUT/pmc $OUT/pmc.json "dataset histograms, tools/bench_hist.py --steps 3 --warmup 1 (1e8 rows)"
