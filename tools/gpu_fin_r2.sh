set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/fin3
mkdir -p $OUT
bash tools/gpu_pmc_r2.sh fin3_pmc || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; echo "ROCPROF FAILED"; exit 1; }
for w in c4 c5; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline --no-secondary --steps 5 --warmup 2 > $OUT/bench_$w.log 2>&1 || { tail -5 $OUT/bench_$w.log; echo "$w failed"; exit 1; }
done
echo fin3 ok
