#!/bin/bash
# Round 4: sieve parity (both level-1 shapes), then C3 bench with 512- and
# 1,024-thread sieve workgroups (TAG = $1); stops at the first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r4a}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_sieve.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_sieve.log 2>&1 || { echo "SIEVE TESTS FAILED"; tail -30 $OUT/pytest_sieve.log; exit 1; }
tail -2 $OUT/pytest_sieve.log
for TH in 512 1024 512; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-api --sieve-threads $TH > $OUT/bench_t$TH.json 2> $OUT/bench_t$TH.err || { echo "BENCH $TH FAILED"; tail -20 $OUT/bench_t$TH.err; exit 1; }
  python3 - $OUT/bench_t$TH.json $TH <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], "C3 ms/step %.3f" % r["ms_per_step"], {k: round(v["ms"], 3) for k, v in r["kernels"].items() if v["ms"] > 0.03})
s = r.get("secondary")
if s:
    print(sys.argv[2], "C2 ms/step %.3f" % s["ms_per_step"], {k: round(v["ms"], 3) for k, v in s["kernels"].items() if v["ms"] > 0.03})
PY
done
echo "r4a ok"
