#!/bin/bash
# Round 6: per-XCD contract times of 16 back-to-back C2 launches with the workgroups' starts staggered within each
# XCD (trace_stag_variant.sh) against the plain trace variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
: > gpurun_out/r06_trace_stagger.txt
for v in trace trace_stag; do
  SMC_LIB_PATH=tools/micro/v/libsmc_$v.so timeout -k 10 120 python tools/kprof_step.py --config c2 --iters 16 --dynamic --trace-timed gpurun_out/ts_$v.npy >> gpurun_out/r06_trace_stagger.txt 2>&1 || exit 1
done
grep -v amdgpu.ids gpurun_out/r06_trace_stagger.txt
