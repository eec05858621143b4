#!/bin/bash
# k_sieve_l1 across processes on one box: default allocator vs expandable segments, 3 processes each, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-l1spread}
mkdir -p $OUT
for i in 1 2 3; do
  for mode in default expandable; do
    if [ $mode = expandable ]; then export PYTORCH_HIP_ALLOC_CONF=expandable_segments:True; else unset PYTORCH_HIP_ALLOC_CONF; fi
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-api > $OUT/$mode.$i.json 2> $OUT/$mode.$i.err || { echo "run $mode $i failed"; tail -5 $OUT/$mode.$i.err; exit 1; }
    python3 -c "
import json
r=json.loads([l for l in open('$OUT/$mode.$i.json') if l.startswith('{')][-1])
print('$mode $i', 'ms %.3f' % r['ms_per_step'], 'L1 %.3f' % r['kernels']['k_sieve_l1']['ms'], 'L2 %.3f' % r['kernels']['k_scatter_l2']['ms'], 'bucket %.3f' % r['kernels']['k_bucket_bound']['ms'], flush=True)
"
  done
done
