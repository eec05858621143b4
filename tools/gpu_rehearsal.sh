#!/bin/bash
# 2-rank gloo rehearsals on one GPU (both ranks share the card): C4 and C3 shards, the
# library's default privacy_id_sharding="verify" timed once per run (TAG = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-rehearsal}
OUT=gpurun_out/$T
mkdir -p $OUT
export PDP_BENCH_BACKEND=gloo
timeout -k 10 400 python -u bench.py --workload c4 --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c4.json 2> $OUT/c4.err || { echo "c4 failed"; tail -20 $OUT/c4.err; exit 1; }
timeout -k 10 400 python -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline --no-api > $OUT/c3.json 2> $OUT/c3.err || { echo "c3 failed"; tail -20 $OUT/c3.err; exit 1; }
python3 - $OUT <<'PY'
import json, sys
for w in ("c4", "c3"):
    r = json.loads([l for l in open(f"{sys.argv[1]}/{w}.json") if l.startswith("{")][-1])
    print(w, "ms/step %.2f" % r["ms_per_step"], "verify", r.get("privacy_id_verify"))
PY
