#!/bin/bash
# Times the contract kernel (C2, hw math, padded pitch) for each named variant library
# tools/micro/libsmc_<name>.so, store-all and terminal-only.
# Usage: run_decomp.sh name[,extra kprof args] ...   e.g. run_decomp.sh s4 s4nocf,--unsliced
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
for spec in "$@"; do
  name=${spec%%,*}
  extra=""
  [ "$name" != "$spec" ] && extra=${spec#*,}
  for store in all terminal; do
    SMC_LIB_PATH=$PWD/tools/micro/libsmc_$name.so timeout -k 10 120 python tools/kprof.py --math hw --store $store --iters 10 $extra 2>&1 | grep -v amdgpu.ids || exit $?
  done
done
