#!/bin/bash
# Round-3 kernel profile of one bench workload: rocprofv3 kernel trace +
# stats, then separate --pmc passes (MI355X_MICROARCH.md: one TCC group per
# pass; <= 8 SQ counters per pass), each under its own time limit; stops at
# the first failure.  tools/pmc_summary.py -> $OUT/<W>_pmc.json.
# Usage: bash tools/gpu_prof_r3.sh TAG [WORKLOAD] [extra bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-prof_r3}
W=${2:-c3}
shift 2
EXTRA="$@"
OUT=gpurun_out/$TAG
mkdir -p $OUT
declare -A ROWS=([c3]=1000000000 [c2]=100000000 [c4]=125000000 [c5]=625000000 [hist]=100000000)
BENCH="python -u bench.py --workload $W --steps 2 --warmup 1 --no-cpu-baseline --no-secondary --no-api $EXTRA"
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/$W/trace -o run --output-format csv -- $BENCH > $OUT/${W}_trace.log 2>&1 || { echo "trace pass failed"; tail -5 $OUT/${W}_trace.log; exit 1; }
SQ1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
SQ2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM"
i=0
for C in FETCH_SIZE WRITE_SIZE "$SQ1" "$SQ2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $C -d $OUT/$W/pmc$i -o run --output-format csv -- $BENCH > $OUT/${W}_pmc$i.log 2>&1 || { echo "PMC pass $i ($C) failed"; tail -5 $OUT/${W}_pmc$i.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT/$W $OUT/${W}_pmc.json "$W n=${ROWS[$W]} " $OUT/${W}_pmc1.log || exit 1
echo "prof ok"
