#!/bin/bash
# MFMA utilisation of the network kernels: SQ_VALU_MFMA_BUSY_CYCLES (cycles, summed over the chip's
# SIMDs), SQ_BUSY_CYCLES and GRBM_GUI_ACTIVE per dispatch of tools/kprof_net.py; one --pmc pass
# per spec (arch:compute).  CSVs into gpurun_out/pmcnet_<arch>_<compute>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for spec in "$@"; do
  arch=${spec%%:*}
  compute=${spec##*:}
  out=gpurun_out/pmcnet_${arch}_${compute}
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    -d "$out" -o run --output-format csv -- python3 tools/kprof_net.py --arch "$arch" --compute "$compute" --iters 5 \
    > "$out.log" 2>&1 || exit $?
  grep "us/step" "$out.log"
done
