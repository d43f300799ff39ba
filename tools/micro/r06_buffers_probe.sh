#!/bin/bash
# Round 6: does the C2 launch's speed follow its path buffer?  Serialised launches on one buffer vs rotating over
# four buffers (one stream) vs four lanes in flight, each traced (per-XCD contract times and shader clock).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export SMC_LIB_PATH=tools/micro/v/libsmc_trace.so
o=gpurun_out/r06_buffers_probe.txt; : > $o
for rep in 1 2; do
  timeout -k 10 120 python tools/kprof_step.py --config c2 --iters 16 --dynamic --trace-timed gpurun_out/tb_one_$rep.npy >> $o 2>&1 || exit 1
  timeout -k 10 120 python tools/kprof_step.py --config c2 --iters 16 --dynamic --lanes 4 --one-stream --trace-timed gpurun_out/tb_rot_$rep.npy >> $o 2>&1 || exit 1
  timeout -k 10 120 python tools/kprof_step.py --config c2 --iters 16 --dynamic --lanes 4 --trace-timed gpurun_out/tb_l4_$rep.npy >> $o 2>&1 || exit 1
done
grep -v amdgpu.ids $o
