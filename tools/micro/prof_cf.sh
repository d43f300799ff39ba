#!/bin/bash
# Per-kernel durations (rocprofv3 kernel trace) of the C2 training launch for the in-tree library
# and tools/micro/libsmc_<name>.so variants; summaries into gpurun_out/prof_<name>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for lib in spectralmc_amd/libspectralmc_hip.so tools/micro/libsmc_*.so; do
  [ -f "$lib" ] || continue
  name=$(basename "$lib" .so)
  SMC_LIB_PATH=$PWD/$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$name -o run \
    -- python3 tools/kprof.py --unsliced --math hw --store all --iters 10 > gpurun_out/prof_$name.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/prof_$name.log | tail -1
  python3 tools/rocpd_stats.py gpurun_out/prof_$name/run_results.db paths_kernel cf_kernel contract_kernel
done
