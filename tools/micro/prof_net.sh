#!/bin/bash
# Per-kernel durations (rocprofv3 kernel trace) of the fused network step for the C2 / H256 / C3
# networks on the VALU and MFMA kernels; summaries into gpurun_out/net_<arch>_<compute>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
for spec in "$@"; do
  arch=${spec%%:*}
  compute=${spec##*:}
  out=gpurun_out/net_${arch}_${compute}
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$out" -o run \
    -- python3 tools/kprof_net.py --arch "$arch" --compute "$compute" > "$out.log" 2>&1 || exit $?
  grep "us/step" "$out.log"
  python3 tools/rocpd_stats.py "$out/run_results.db" | grep -v -E "elementwise|fill|copy|Memcpy" | head -8
done
