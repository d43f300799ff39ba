#!/bin/bash
# A/B driver for tools/micro/make_variant.py libraries on the GPU box: each variant runs
# ${AB_SCRIPT:-tools/kprof_step.py} ARGS with SMC_LIB_PATH=tools/micro/v/libsmc_<name>.so ("default": the in-tree
# library), interleaved over two passes.  Usage: tools/micro/ab.sh OUT.txt "kprof_step args" name ...
set -u
out=$1; args=$2; shift 2
mkdir -p "$(dirname "$out")"
for rep in 1 2; do
  for name in "$@"; do
    if [ "$name" = default ]; then lib=spectralmc_amd/libspectralmc_hip.so; else lib=tools/micro/v/libsmc_$name.so; fi
    echo -n "$name: " >> "$out"
    SMC_LIB_PATH=$lib timeout -k 10 120 python "${AB_SCRIPT:-tools/kprof_step.py}" $args 2>/dev/null | grep -v amdgpu.ids >> "$out" || exit 1
  done
done
