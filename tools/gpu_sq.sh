#!/bin/bash
# SQ counter passes (LDS / VALU / waits) over a short bench run of one library
# variant.  Usage: bash tools/gpu_sq.sh TAG LIB.so
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-sq}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PIPELINEDP_AMD_LIB=$PWD/${2:-pipelinedp_amd/lib/libpipelinedp_amd.so}
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS" "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C -d $OUT/p$i -o run --output-format csv -- python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --no-api > $OUT/p$i.log 2>&1 || { echo "PMC pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT $OUT/sq.json "$TAG" > /dev/null
python3 - $OUT/sq.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["kernels"]
for k in ("k_bucket_bound", "k_scatter_l1", "k_scatter_l2", "k_part_hist", "k_range_reduce"):  # (pmc_summary maps the _local kernels)
    if k in d:
        print(k, {c: "%.4g" % v for c, v in sorted(d[k]["counters_avg_per_launch"].items())})
PY
