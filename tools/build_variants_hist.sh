#!/bin/bash
# A/B variants of pdp_hist.hip (compile-time knobs) into abv/, the other sources
# compiled once (build/abv_common/); usage: name:flags ...
set -e
cd "$(dirname "$0")/.."
mkdir -p abv build/abv_common
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -I include"
common=()
for src in pipelinedp_amd/csrc/*.hip; do
  [ "$(basename $src)" = pdp_hist.hip ] && continue
  obj=build/abv_common/h_$(basename $src .hip).o
  if [ ! -f $obj ] || [ $src -nt $obj ] || [ pipelinedp_amd/csrc/pdp_internal.h -nt $obj ]; then
    /opt/rocm/bin/hipcc $FLAGS -c $src -o $obj &
  fi
  common+=($obj)
done
wait
# a variant named NAME builds abv_src/NAME/pdp_hist.hip instead when that file
# exists (e.g. an older revision: git show REV:pipelinedp_amd/csrc/pdp_hist.hip)
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  [ "$name" = "$spec" ] && flags=""
  src=pipelinedp_amd/csrc/pdp_hist.hip
  if [ -f abv_src/$name/pdp_hist.hip ]; then
    cp pipelinedp_amd/csrc/pdp_internal.h abv_src/$name/
    src=abv_src/$name/pdp_hist.hip
  fi
  ( /opt/rocm/bin/hipcc $FLAGS $flags -I include -c $src -o build/abv_common/hist_$name.o && \
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o abv/$name.so build/abv_common/hist_$name.o "${common[@]}" ) &
done
wait
ls -la abv
