#!/bin/bash
# Final-tree profiles (TAG = $1, default prof): per workload a rocprofv3
# kernel-trace summary (20 timed steps) and the FETCH_SIZE / WRITE_SIZE PMC
# passes (one counter per run, MI355X_MICROARCH.md "HBM"), summarised by
# tools/pmc_summary.py into $OUT/<w>_pmc.json for bench.py's roofline join.
# WORKLOADS="c3 c2 c4 c5 hist" by default.  Every GPU step has a time limit;
# the first failure ends the script.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-prof}
mkdir -p $OUT
for W in ${WORKLOADS:-c3 c2 c4 c5 hist}; do
  case $W in
    c3) N=1000000000; ARGS="--no-secondary --no-api" ;;
    c2) N=100000000; ARGS="--workload c2 --no-api" ;;
    c4) N=125000000; ARGS="--workload c4" ;;
    c5) N=625000000; ARGS="--workload c5" ;;
    hist) N=100000000; ARGS="--workload hist" ;;
  esac
  mkdir -p $OUT/$W
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/$W/stats -o run --output-format csv -- python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline $ARGS > $OUT/$W/stats.log 2>&1 || { tail -20 $OUT/$W/stats.log; echo "ROCPROF $W FAILED"; exit 1; }
  find $OUT/$W/stats -name "*kernel_stats.csv" -exec cp {} $OUT/${W}_kernel_stats.csv \;
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $C -d $OUT/$W/pmc/$C -o run --output-format csv -- python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline $ARGS > $OUT/$W/pmc_$C.log 2>&1 || { tail -20 $OUT/$W/pmc_$C.log; echo "PMC $W $C FAILED"; exit 1; }
  done
  python3 tools/pmc_summary.py $OUT/$W/pmc $OUT/${W}_pmc.json "$W n=$N bench.py --steps 3 --warmup 1 $ARGS" $OUT/$W/pmc_FETCH_SIZE.log || exit 1
  echo "$W profiled"
done
