set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -m gpu > gpurun_out/r1_pytest.log 2>&1; rc=$?
tail -30 gpurun_out/r1_pytest.log
if [ $rc -ne 0 ]; then echo "PYTEST FAILED rc=$rc"; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r1_bench.log 2>&1 && cat gpurun_out/r1_bench.log
