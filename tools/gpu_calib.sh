#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on known line counts (tools/fetch_calib.hip)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-calib}
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $OUT/f -o run --output-format csv -- ./tools/fetch_calib > $OUT/f.log 2>&1 || { echo "FETCH pass failed"; tail -5 $OUT/f.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $OUT/w -o run --output-format csv -- ./tools/fetch_calib > $OUT/w.log 2>&1 || { echo "WRITE pass failed"; tail -5 $OUT/w.log; exit 1; }
python3 tools/fetch_calib.py $OUT $OUT/calib.json
