#!/bin/bash
# Builds A/B variants of the library (compile-time knobs) into abv/
# for tools/gpu_variants.sh; the product library is built by __graft_entry__.build().
# Only pdp_bound.hip is recompiled per variant; the other sources are compiled
# once (build/abv_common/) and linked into every variant.
set -e
cd "$(dirname "$0")/.."
mkdir -p abv build/abv_common
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -munsafe-fp-atomics -I include"
common=()
for src in pipelinedp_amd/csrc/*.hip; do
  [ "$(basename $src)" = pdp_bound.hip ] && continue
  obj=build/abv_common/$(basename $src .hip).o
  if [ ! -f $obj ] || [ $src -nt $obj ] || [ pipelinedp_amd/csrc/pdp_internal.h -nt $obj ] || [ include/pipelinedp_amd.h -nt $obj ]; then
    /opt/rocm/bin/hipcc $FLAGS -c $src -o $obj &
  fi
  common+=($obj)
done
wait
# a variant named NAME builds abv_src/NAME/pdp_bound.hip instead when that file
# exists (e.g. an older revision: git show REV:pipelinedp_amd/csrc/pdp_bound.hip)
build() {
  local src=pipelinedp_amd/csrc/pdp_bound.hip
  if [ -f abv_src/$1/pdp_bound.hip ]; then
    cp pipelinedp_amd/csrc/pdp_internal.h abv_src/$1/
    src=abv_src/$1/pdp_bound.hip
  fi
  /opt/rocm/bin/hipcc $FLAGS "${@:2}" -c $src -o build/abv_common/bound_$1.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o abv/$1.so build/abv_common/bound_$1.o "${common[@]}"
}
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  [ "$name" = "$spec" ] && flags=""
  build $name $flags &
done
wait
ls -la abv
