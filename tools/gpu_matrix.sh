#!/bin/bash
# Runs bench.py once per line of a matrix file ("name|bench args"), each under
# its own time limit, and prints ms/step plus the kernels above 0.03 ms;
# stops at the first failure.  Usage: bash tools/gpu_matrix.sh TAG MATRIX_FILE
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-matrix}
mkdir -p $OUT
while IFS='|' read -r name bargs; do
  [ -z "$name" ] && continue
  case "$name" in \#*) continue;; esac
  timeout -k 10 300 python -u bench.py --no-cpu-baseline $bargs > $OUT/$name.json 2> $OUT/$name.err || { echo "BENCH $name FAILED"; tail -20 $OUT/$name.err; exit 1; }
  python3 - $OUT/$name.json $name <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
bp = r.get("bound_plan") or {}
st = bp.get("stats") or {}
print(sys.argv[2], "ms/step %.3f" % r["ms_per_step"], "plan", {k: bp.get(k) for k in ("sieve", "band", "merge", "key_format", "sieve_threads") if k in bp},
      {k: st[k] for k in ("rows_partitioned", "band_rows", "unresolved_ids", "unresolved2_ids") if k in st},
      {k: round(v["ms"], 3) for k, v in r["kernels"].items() if v["ms"] * v.get("launches_per_step", 1) > 0.03}, flush=True)
s = r.get("secondary")
if s:
    print(sys.argv[2], "C2 ms/step %.3f" % s["ms_per_step"], {k: round(v["ms"], 3) for k, v in s["kernels"].items() if v["ms"] > 0.03})
PY
done < $2
echo "matrix ok"
