#!/bin/bash
# pytest of the bounding kernels (all key formats), then C4 / C5 with the abv variants (TAG = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4e}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_sieve.py tests/test_gpu_scale.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for W in c5 c4; do
for so in abv/*.so; do
  v=$(basename $so .so)
  PIPELINEDP_AMD_LIB=$PWD/$so timeout -k 10 300 python -u bench.py --workload $W --steps 5 --warmup 2 --no-cpu-baseline > $OUT/$W.$v.json 2> $OUT/$W.$v.err || { echo "$W $v failed"; tail -5 $OUT/$W.$v.err; exit 1; }
  python3 - $OUT/$W.$v.json $W.$v <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], "ms/step %.3f" % r["ms_per_step"], {k: round(v["ms"] * v.get("launches_per_step", 1), 3) for k, v in r["kernels"].items() if v["ms"] * v.get("launches_per_step", 1) > 0.05}, flush=True)
PY
done
done
