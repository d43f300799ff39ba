#!/bin/bash
# Times the contract kernel of the in-tree library and of each prebuilt variant
# (tools/micro/libsmc_*.so) at contiguous (pitch 0) and padded (pitch -1) path rows.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for lib in spectralmc_amd/libspectralmc_hip.so tools/micro/libsmc_*.so; do
  [ -f "$lib" ] || continue
  for store in all terminal; do
    for pitch in 0 -1; do
      SMC_LIB_PATH=$PWD/$lib timeout -k 10 120 python tools/kprof.py --math hw --store $store --iters 10 --pitch $pitch || exit $?
    done
  done
done
