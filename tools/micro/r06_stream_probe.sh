#!/bin/bash
# Round 6: one C2 launch at a time on torch's current stream vs on a created stream (default / high priority), two
# passes; then per-XCD traces of 16 launches on each (trace variant).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r06_stream_probe.txt; : > $o
for rep in 1 2; do
  for st in current created high; do
    for dyn in "" "--dynamic"; do
      echo -n "[$st $dyn] " >> $o
      timeout -k 10 120 python tools/kprof_step.py --config c2 --iters 16 --stream $st $dyn 2>/dev/null | grep -v amdgpu.ids >> $o || exit 1
    done
  done
done
for st in current created; do
  SMC_LIB_PATH=tools/micro/v/libsmc_trace.so timeout -k 10 120 python tools/kprof_step.py --config c2 --iters 16 --dynamic --stream $st --trace-timed gpurun_out/tstream_$st.npy > /dev/null 2>&1 || exit 1
done
sed -E 's/c2 normalize pitch=66560 (B=[0-9]+).*resident_kernel: ([0-9.]+ ms\/step).*/\1 \2/' $o
