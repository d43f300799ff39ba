#!/bin/bash
# A/B of resident_kernel builds at C2 (hw, store all): in-tree library vs tools/micro/libsmc_<name>.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
run() { SMC_LIB_PATH=$PWD/$1 timeout -k 10 150 python tools/kprof.py --unsliced --math hw --store all "${@:2}" || exit $?; }
for rep in 1 2 3; do
  for lib in spectralmc_amd/libspectralmc_hip.so tools/micro/libsmc_*.so; do
    [ -f "$lib" ] || continue
    run "$lib" --iters 20
  done
done
