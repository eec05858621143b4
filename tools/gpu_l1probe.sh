#!/bin/bash
# level 1 alone for every abv/*.so, ROUNDS interleaved passes (TAG = $1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-l1probe}
mkdir -p $OUT
rocm-smi --showmeminfo vram > $OUT/smi.txt 2>&1 || true
for pass in $(seq 1 ${ROUNDS:-2}); do
for so in abv/*.so; do
  v=$(basename $so .so)
  PIPELINEDP_AMD_LIB=$PWD/$so timeout -k 10 120 python -u tools/l1_probe.py --tag $v.$pass > $OUT/$v.$pass.log 2>&1 || { echo "variant $v failed"; tail -5 $OUT/$v.$pass.log; exit 1; }
  grep '^{' $OUT/$v.$pass.log
done
done
