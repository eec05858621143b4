#!/bin/bash
# Builds A/B variants of the library (compile-time knobs) into abv/
# for tools/gpu_variants.sh; the product library is built by __graft_entry__.build().
set -e
cd "$(dirname "$0")/.."
mkdir -p abv
build() {
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -munsafe-fp-atomics -I include "${@:2}" \
    -o abv/$1.so pipelinedp_amd/csrc/*.hip
}
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  [ "$name" = "$spec" ] && flags=""
  build $name $flags &
done
wait
ls -la abv
