#!/bin/bash
# PMC passes (one counter group per run) over a short bench run (TAG = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for C in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY"; do
  N=$(echo $C | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/$N -o run --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/$N.log 2>&1 || { echo "PMC pass $C failed"; exit 1; }
done
for f in $(find $OUT -name "*counter_collection.csv"); do echo "== $f"; python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    name = r.get("Kernel_Name", "")[:60]
    agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    if "pdp" not in k: continue
    print(k, {c: sum(v) / len(v) for c, v in d.items()})
PY
done
