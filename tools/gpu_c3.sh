#!/bin/bash
# GPU: C3 bench (1e9 Zipf rows) summarised (TAG = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-c3}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u bench.py --workload c3 --steps 5 --warmup 2 > gpurun_out/$TAG/bench_c3.log 2>&1 || { tail -5 gpurun_out/$TAG/bench_c3.log; exit 1; }
python3 - gpurun_out/$TAG/bench_c3.log <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("C3 ms/step %.3f" % r["ms_per_step"], "rows/s %.3g" % r["value"], {k: round(v, 3) for k, v in r["kernel_ms"].items() if v > 0.05})
PY
