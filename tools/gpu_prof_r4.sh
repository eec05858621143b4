#!/bin/bash
# Round-4 profiles of the final tree: tools/gpu_prof_r3.sh (kernel trace + stats, then
# FETCH_SIZE / WRITE_SIZE / two SQ passes) for each workload named (TAG = $1, then workloads)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; shift
for W in "$@"; do
  case $W in
    c3) X="--no-secondary" ;;
    *) X="" ;;
  esac
  bash tools/gpu_prof_r3.sh $T $W $X || exit 1
done
