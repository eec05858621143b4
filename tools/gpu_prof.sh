#!/bin/bash
# rocprofv3 kernel-trace summary of bench.py (tag = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-prof}
mkdir -p gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG -o run --output-format csv -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$TAG/bench.log 2>&1
rc=$?
tail -3 gpurun_out/$TAG/bench.log
find gpurun_out/$TAG -name "*stats*" | head
exit $rc
