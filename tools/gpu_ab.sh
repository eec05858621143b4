#!/bin/bash
# A/B of abv/*.so: parity of variant $PARITY (default: every variant) on the
# sieve tests, then ROUNDS interleaved bench passes (TAG = $1; bench flags in $BENCH_ARGS)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-ab}
OUT=gpurun_out/$T
mkdir -p $OUT
rocm-smi --showclocks --showpower --showmemuse --showmeminfo vram > $OUT/smi.txt 2>&1 || true
[ -x tools/stream_bench ] && { timeout -k 10 120 tools/stream_bench > $OUT/stream.txt 2>&1 || true; }
for so in abv/*.so; do
  v=$(basename $so .so)
  if [ -n "$PARITY" ] && [ "$PARITY" != "$v" ]; then continue; fi
  if [ -n "$PARITY_TESTS" ]; then
    PIPELINEDP_AMD_LIB=$PWD/$so timeout -k 10 400 python -u -m pytest $PARITY_TESTS -x -q --timeout 200 --timeout-method thread > $OUT/pytest_$v.log 2>&1 || { echo "PYTEST FAILED ($v)"; tail -40 $OUT/pytest_$v.log; exit 1; }
    echo "parity $v: $(tail -1 $OUT/pytest_$v.log)"
  fi
done
ROUNDS=${ROUNDS:-3} bash tools/gpu_variants.sh $T/bench
