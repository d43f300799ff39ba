#!/bin/bash
# Builds decomposition / tuning variants of libspectralmc_hip.so into tools/micro/libsmc_<name>.so
# (CPU side, before a gpurun call).  Usage: tools/micro/build_variants.sh name:"-DFLAG ..." ...
set -eu
cd "$(dirname "$0")/../../spectralmc_amd/csrc"
OUT=../../tools/micro
for spec in "$@"; do
  name=${spec%%:*}
  flags=${spec#*:}
  [ "$flags" = "$spec" ] && flags=""
  mkdir -p "build/v_$name"
  for src in capi sobol gbm cvnn cvnn_mfma basket; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -fvisibility=hidden -munsafe-fp-atomics \
      $flags -c $src.hip -o "build/v_$name/$src.o" &
  done
  for j in $(jobs -p); do wait $j || { echo "build failed: $name"; exit 1; }; done
  /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "$OUT/libsmc_$name.so" build/v_$name/*.o
  echo "built $OUT/libsmc_$name.so ($flags)"
done
