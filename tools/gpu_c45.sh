#!/bin/bash
# C4 and C5 bench lines per library variant in build/variants (TAG = $1).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-c45}
mkdir -p $OUT
for so in build/variants/*.so; do
  v=$(basename $so .so)
  for w in c4 c5; do
    PIPELINEDP_AMD_LIB=$PWD/$so timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --no-secondary --no-api --steps 5 --warmup 2 > $OUT/${v}_$w.log 2>&1 || { echo "$v $w failed"; tail -5 $OUT/${v}_$w.log; exit 1; }
    python3 -c "
import json
r=json.loads([l for l in open('$OUT/${v}_$w.log') if l.startswith('{')][-1])
print('$v', '$w', round(r['ms_per_step'],3), {k:round(v['ms'],3) for k,v in r['kernels'].items() if v['ms']>0.1})
"
  done
done
