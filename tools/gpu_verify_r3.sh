#!/bin/bash
# the library's default privacy_id_sharding="verify" at
# U = 1e8 (C4 / C5 shape), rehearsed with two gloo ranks sharing one MI355X:
# each rank holds C4's 1.25e8 rows per GPU with 5e7 privacy ids of its own
# (rank r's ids are r * U + k), so the check sees 1e8 distinct ids; the bench
# runs verify once before timing and reports privacy_id_verify_ms (rank 0's
# wall time: torch.unique + one all-to-all of 8 B per id over gloo, i.e. via
# host memory -- RCCL moves the same bytes over xGMI).  Then the C3 2-rank
# rehearsal the same way.  Each step under its own time limit.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-verify_r3}
mkdir -p $OUT
export PDP_BENCH_BACKEND=gloo
timeout -k 10 500 python -u bench.py --gpus 2 --workload c4 --privacy-ids 50000000 --steps 3 --warmup 1 \
  --no-cpu-baseline > $OUT/c4_u1e8_2ranks_gloo.json 2> $OUT/c4_u1e8_2ranks_gloo.err || { echo "c4 rehearsal failed"; tail -20 $OUT/c4_u1e8_2ranks_gloo.err; exit 1; }
timeout -k 10 400 python -u bench.py --gpus 2 --workload c3 --steps 5 --warmup 2 --no-cpu-baseline --no-api \
  > $OUT/c3_2ranks_gloo.json 2> $OUT/c3_2ranks_gloo.err || { echo "c3 rehearsal failed"; tail -20 $OUT/c3_2ranks_gloo.err; exit 1; }
echo "verify rehearsal ok"
