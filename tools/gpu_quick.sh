#!/bin/bash
# GPU: all -m gpu tests, then one bench run summarised (TAG = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-quick}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.log 2>&1
rc=$?
tail -3 gpurun_out/$TAG/pytest.log
if [ $rc -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error" gpurun_out/$TAG/pytest.log | head -20; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/$TAG/bench.log 2>&1 || { tail -5 gpurun_out/$TAG/bench.log; exit 1; }
python3 - gpurun_out/$TAG/bench.log <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("ms/step %.3f" % r["ms_per_step"], {k: round(v, 3) for k, v in r["kernel_ms"].items() if v > 0.004})
PY
