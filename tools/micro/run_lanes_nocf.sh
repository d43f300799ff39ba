#!/bin/bash
# C2 MC part with 2 lanes (tools/kprof_step.py --lanes 2 --dynamic): in-tree library vs the no-CF build
set -u
out=$1
for rep in 1 2; do
  for lib in spectralmc_amd/libspectralmc_hip.so tools/micro/libsmc_nocf.so; do
    echo -n "$lib: " >> "$out"
    SMC_LIB_PATH=$lib timeout -k 10 120 python tools/kprof_step.py --config c2 --iters 20 --lanes 2 --dynamic 2>/dev/null | grep -v amdgpu.ids >> "$out" || exit 1
  done
done
