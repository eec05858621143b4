set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r6n
mkdir -p $OUT
PIPELINEDP_AMD_LIB=$PWD/abv/b_t2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_sieve.py tests/test_gpu_kernels.py "tests/test_gpu_scale.py::test_c4_shape_matches_oracle_with_selection_and_noise" tests/test_gpu_scale.py::test_c2_full_scale_sampling_matches_oracle -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for pass in 1 2; do for v in a_t1 b_t2; do
  PIPELINEDP_AMD_LIB=$PWD/abv/$v.so timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-api > $OUT/$v.c3.$pass.log 2>&1 || exit 1
  PIPELINEDP_AMD_LIB=$PWD/abv/$v.so timeout -k 10 300 python -u bench.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/$v.c4.$pass.log 2>&1 || exit 1
  python3 - $OUT/$v.c3.$pass.log $OUT/$v.c4.$pass.log $v.$pass <<'PY'
import json, sys
a = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
b = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
k = lambda r, n: round(r["kernels"].get(n, {}).get("ms", 0), 3)
print(sys.argv[3], "C3 %.3f bucket %.3f L1 %.3f | C2 %.3f bucket %.3f | C4 %.3f bucket %.3f" % (a["ms_per_step"], k(a, "k_bucket_bound"), k(a, "k_sieve_l1"), a["secondary"]["ms_per_step"], k(a["secondary"], "k_bucket_bound"), b["ms_per_step"], k(b, "k_bucket_bound")), flush=True)
PY
done; done
