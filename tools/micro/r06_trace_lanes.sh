#!/bin/bash
# Round 6: per-workgroup traces (tools/micro/trace_variant.sh) of one C2 launch alone and of 4 launches on 4 lanes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export SMC_LIB_PATH=tools/micro/v/libsmc_trace.so
timeout -k 10 120 python tools/kprof_step.py --config c2 --iters 10 --trace gpurun_out/trace_alone.npy > gpurun_out/r06_trace_alone.txt 2>&1 || exit 1
timeout -k 10 120 python tools/kprof_step.py --config c2 --iters 20 --lanes 4 --dynamic --trace gpurun_out/trace_lanes4.npy > gpurun_out/r06_trace_lanes4.txt 2>&1 || exit 1
cat gpurun_out/r06_trace_alone.txt gpurun_out/r06_trace_lanes4.txt | grep -v amdgpu.ids
