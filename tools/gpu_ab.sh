#!/bin/bash
# GPU: parity tests, then bench with each key format (TAG = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
tail -5 $OUT/pytest.log
if [ $rc -ne 0 ]; then echo "PYTEST FAILED rc=$rc"; grep -E "^(FAILED|ERROR)|Error" $OUT/pytest.log | head -20; exit $rc; fi
for KF in 2 1; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --key-format $KF > $OUT/bench_k$KF.log 2>&1 || { echo "BENCH k$KF FAILED"; tail -5 $OUT/bench_k$KF.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/bench_k$KF.log').read().strip().splitlines()[-1]); print('k$KF', round(d['ms_per_step'],3), 'ms', {k: round(v,3) for k,v in d['kernel_ms'].items() if v > 0.02})"
done
