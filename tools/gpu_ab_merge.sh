#!/bin/bash
# C4 / C5 merge A/B: parity of abv/$PARITY.so on the merge tests, then C4 and C5 bench passes per variant (TAG = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-abm}
OUT=gpurun_out/$T
mkdir -p $OUT
if [ -n "$PARITY" ]; then
  PIPELINEDP_AMD_LIB=$PWD/abv/$PARITY.so timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_scale.py ${PARITY_FILES:-} -k "${PARITY_K:-two_level or half_size or range_merge or c4}" -x -q --timeout 250 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -30 $OUT/pytest.log; exit 1; }
  echo "parity $PARITY: $(tail -1 $OUT/pytest.log)"
fi
for pass in $(seq 1 ${ROUNDS:-2}); do
for so in abv/*.so; do
  v=$(basename $so .so)
  for w in ${WORKLOADS:-c4 c5}; do
    PIPELINEDP_AMD_LIB=$PWD/$so timeout -k 10 240 python -u bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline --no-api --no-secondary > $OUT/$v.$w.$pass.log 2>&1 || { echo "variant $v $w failed"; tail -5 $OUT/$v.$w.$pass.log; exit 1; }
    python3 - $OUT/$v.$w.$pass.log $v.$w.$pass <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], "ms/step %.3f" % r["ms_per_step"], {k: round(v["ms"], 3) for k, v in r["kernels"].items() if k.startswith(("k_split", "k_fine", "k_range", "k_sieve_l1"))})
PY
  done
done
done
