#!/bin/bash
# A/B of the training path/CF kernels at C2 (hw, store all): in-tree library (paths_kernel +
# cf_kernel) at 4 / 3 / 2 resident paths workgroups per CU vs tools/micro/libsmc_<name>.so builds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
run() { SMC_LIB_PATH=$PWD/$1 timeout -k 10 150 python tools/kprof.py --unsliced --math hw --store all "${@:2}" || exit $?; }
for rep in 1 2; do
  run spectralmc_amd/libspectralmc_hip.so --iters 20
  SMC_PATHS_LDS_KB=45 run spectralmc_amd/libspectralmc_hip.so --iters 20
  SMC_PATHS_LDS_KB=60 run spectralmc_amd/libspectralmc_hip.so --iters 20
  for lib in tools/micro/libsmc_*.so; do
    [ -f "$lib" ] || continue
    run "$lib" --iters 20
  done
done
run spectralmc_amd/libspectralmc_hip.so --iters 3 --B 2048 --N 1024
run tools/micro/libsmc_fused.so --iters 3 --B 2048 --N 1024
