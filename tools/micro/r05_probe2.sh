#!/bin/bash
# round 5, GPU call 2: row-pitch sweep of the store order (storebench8 sweep) and the C2 launch at several pitches
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05p2; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 150 tools/micro/v/storebench8 sweep > $O/storebench8_sweep.txt 2>&1 || exit $?
for rep in 1 2; do
  for p in 66560 69632 73728 74752 77824 81920 90112; do
    timeout -k 10 120 python tools/kprof_step.py --config c2 --iters 10 --pitch $p 2>/dev/null | grep -v amdgpu.ids >> $O/c2_pitch.txt || exit $?
  done
done
