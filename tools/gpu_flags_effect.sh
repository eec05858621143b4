#!/bin/bash
# C3 headline: bench.py defaults vs --no-cpu-baseline --no-secondary --no-api, interleaved x2 on one box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-flags}
mkdir -p $OUT
for i in 1 2; do
  for mode in default bare; do
    X=""; [ $mode = bare ] && X="--no-cpu-baseline --no-secondary --no-api"
    timeout -k 10 400 python -u bench.py $X > $OUT/$mode.$i.json 2> $OUT/$mode.$i.err || { echo "run $mode $i failed"; tail -5 $OUT/$mode.$i.err; exit 1; }
    python3 -c "
import json
r=json.loads([l for l in open('$OUT/$mode.$i.json') if l.startswith('{')][-1])
print('$mode $i', 'ms %.3f' % r['ms_per_step'], 'L1 %.3f' % r['kernels']['k_sieve_l1']['ms'], flush=True)
"
  done
done
