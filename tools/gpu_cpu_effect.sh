#!/bin/bash
# C3 with and without the in-process CPU baseline before the GPU work, interleaved x2 (expandable segments set by bench.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-cpueffect}
mkdir -p $OUT
for i in 1 2; do
  for mode in withcpu nocpu; do
    X="--no-secondary --no-api"; [ $mode = nocpu ] && X="$X --no-cpu-baseline"
    timeout -k 10 300 python -u bench.py $X > $OUT/$mode.$i.json 2> $OUT/$mode.$i.err || { echo "run $mode $i failed"; tail -5 $OUT/$mode.$i.err; exit 1; }
    python3 -c "
import json
r=json.loads([l for l in open('$OUT/$mode.$i.json') if l.startswith('{')][-1])
print('$mode $i', 'ms %.3f' % r['ms_per_step'], 'L1 %.3f' % r['kernels']['k_sieve_l1']['ms'], 'L2 %.3f' % r['kernels']['k_scatter_l2']['ms'], flush=True)
"
  done
done
