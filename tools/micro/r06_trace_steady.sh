#!/bin/bash
# Round 6: per-workgroup traces of 16 timed C2 launches: one lane (back to back) and four lanes (in flight)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export SMC_LIB_PATH=tools/micro/v/libsmc_trace.so
timeout -k 10 120 python tools/kprof_step.py --config c2 --iters 16 --dynamic --trace-timed gpurun_out/trace_steady_l1.npy > gpurun_out/r06_trace_steady.txt 2>&1 || exit 1
timeout -k 10 120 python tools/kprof_step.py --config c2 --iters 16 --lanes 4 --dynamic --trace-timed gpurun_out/trace_steady_l4.npy >> gpurun_out/r06_trace_steady.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/r06_trace_steady.txt
