#!/bin/bash
# round 5: box CPU share, sieve + abi GPU tests, C3 bench (full line), light-user bench (TAG = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r5k}
OUT=gpurun_out/$T
mkdir -p $OUT
{ nproc; python3 -c "import os; print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))"; cat /sys/fs/cgroup/cpu.max 2>&1; echo "OMP=$OMP_NUM_THREADS"; } > $OUT/cpus.txt 2>&1
rocm-smi --showmeminfo vram > $OUT/smi.txt 2>&1 || true
timeout -k 10 600 python -u -m pytest tests/test_gpu_sieve.py tests/test_abi.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 $OUT/bench.log; exit 1; }
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --small-ids 0.3 --no-cpu-baseline --no-secondary --no-api > $OUT/bench_small.log 2>&1 && timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --small-ids 0.3 --sieve -1 --no-cpu-baseline --no-secondary --no-api > $OUT/bench_small_nosieve.log 2>&1 && timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --share-of 8 --no-cpu-baseline --no-api > $OUT/bench_share8.log 2>&1 || { echo "BENCH small/share FAILED"; exit 1; }
python3 tools/bench_summary.py $OUT/bench.log $OUT/bench_small.log $OUT/bench_small_nosieve.log $OUT/bench_share8.log 2>/dev/null || grep -h '^{' $OUT/bench.log $OUT/bench_small.log | cut -c1-300
