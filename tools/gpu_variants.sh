#!/bin/bash
# Runs the bench once per library variant in abv, in ROUNDS interleaved passes
# (default 2: A B A B, so box drift shows), TAG = $1; extra bench flags in $BENCH_ARGS
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-variants}
mkdir -p $OUT
for pass in $(seq 1 ${ROUNDS:-2}); do
for so in abv/*.so; do
  v=$(basename $so .so)
  PIPELINEDP_AMD_LIB=$PWD/$so timeout -k 10 240 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline $BENCH_ARGS > $OUT/$v.$pass.log 2>&1 || { echo "variant $v failed"; tail -5 $OUT/$v.$pass.log; exit 1; }
  python3 - $OUT/$v.$pass.log $v.$pass <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
r = json.loads(line)
print(sys.argv[2], "C3 ms/step %.3f" % r["ms_per_step"], {k: round(v["ms"] * v.get("launches_per_step", 1), 3) for k, v in r["kernels"].items() if v["ms"] * v.get("launches_per_step", 1) > 0.05}, flush=True)
pl = (r.get("bound_plan") or {}).get("placement") or []
if pl:
    print(sys.argv[2], "placement", pl[0].get("candidates_ms"), "chosen", pl[0].get("chosen"), flush=True)
s = r.get("secondary")
if s:
    print(sys.argv[2], "C2 ms/step %.3f" % s["ms_per_step"], {k: round(v["ms"], 3) for k, v in s["kernels"].items() if v["ms"] > 0.05})
PY
done
done
