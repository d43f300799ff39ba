#!/bin/bash
# Times the contract kernel of each prebuilt workgroup-size variant (tools/micro/libsmc_*.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for lib in tools/micro/libsmc_*.so; do
  for store in all terminal; do
    SMC_LIB_PATH=$PWD/$lib timeout -k 10 120 python tools/kprof.py --math hw --store $store --iters 10 || exit $?
  done
done
