#!/bin/bash
# A/B of the training path/CF kernels at C2 and C3 (hw, store all): in-tree library
# (resident_kernel at C2) vs tools/micro/libsmc_<name>.so builds (split pair, fused contract_kernel).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
run() { SMC_LIB_PATH=$PWD/$1 timeout -k 10 150 python tools/kprof.py --unsliced --math hw --store all "${@:2}" || exit $?; }
for rep in 1 2; do
  for lib in spectralmc_amd/libspectralmc_hip.so tools/micro/libsmc_*.so; do
    [ -f "$lib" ] || continue
    run "$lib" --iters 20
  done
done
run spectralmc_amd/libspectralmc_hip.so --iters 20 --math portable
run tools/micro/libsmc_split.so --iters 20 --math portable
run spectralmc_amd/libspectralmc_hip.so --iters 3 --B 2048 --N 1024
