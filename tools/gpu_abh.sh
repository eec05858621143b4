#!/bin/bash
# histogram A/B: parity of $PARITY on the histogram tests, then ROUNDS bench passes (TAG = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-abh}
OUT=gpurun_out/$T
mkdir -p $OUT
if [ -n "$PARITY" ]; then
  PIPELINEDP_AMD_LIB=$PWD/abv/$PARITY.so timeout -k 10 500 python -u -m pytest tests/test_gpu_histograms.py -x -q --timeout 250 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -30 $OUT/pytest.log; exit 1; }
  echo "parity $PARITY: $(tail -1 $OUT/pytest.log)"
fi
for pass in $(seq 1 ${ROUNDS:-2}); do
for so in abv/*.so; do
  v=$(basename $so .so)
  PIPELINEDP_AMD_LIB=$PWD/$so timeout -k 10 240 python -u bench.py --workload hist --steps 10 --warmup 3 --no-cpu-baseline > $OUT/$v.$pass.log 2>&1 || { echo "variant $v failed"; tail -5 $OUT/$v.$pass.log; exit 1; }
  python3 - $OUT/$v.$pass.log $v.$pass <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], "hist ms/step %.3f" % r["ms_per_step"], {k: round(v["ms"], 3) for k, v in r["kernels"].items() if v["ms"] > 0.05})
PY
done
done
