#!/bin/bash
# C3 with explicit sieve thresholds (t * 2^16; 0 = auto): step time and fix-up statistics (TAG = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-sweep}
OUT=gpurun_out/$T
mkdir -p $OUT
for s in ${SIEVES:-0 8192 6554 12000 0}; do
  timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-api --sieve $s > $OUT/s$s.log 2>&1 || { echo "sieve $s failed"; tail -5 $OUT/s$s.log; exit 1; }
  python3 - $OUT/s$s.log $s <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
st = r["bound_plan"]["stats"]
print("sieve", sys.argv[2], "ms %.3f" % r["ms_per_step"], "t", r["bound_plan"]["sieve"], {k: st[k] for k in ("rows_partitioned", "unresolved_ids", "fixup_rows", "band_rows", "unresolved2_ids", "fixup2_rows")},
      {k: round(v["ms"] * v.get("launches_per_step", 1), 3) for k, v in r["kernels"].items() if v["ms"] * v.get("launches_per_step", 1) > 0.03})
PY
done
