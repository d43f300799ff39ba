#!/bin/bash
# A/B driver for tools/micro variant libraries on the GPU box: each "name" runs tools/kprof_step.py
# (C2 MC part, smc_train_step) with SMC_LIB_PATH=tools/micro/libsmc_<name>.so ("default": the
# in-tree library).  Usage: tools/micro/run_probe.sh OUT.txt name [name ...]
set -u
out=$1; shift
mkdir -p gpurun_out
for name in "$@"; do
  if [ "$name" = default ]; then lib=spectralmc_amd/libspectralmc_hip.so; else lib=tools/micro/libsmc_$name.so; fi
  echo -n "$name: " >> "$out"
  SMC_LIB_PATH=$lib timeout -k 10 120 python tools/kprof_step.py --config c2 --iters 10 2>/dev/null | grep -v amdgpu.ids >> "$out" || exit 1
done
