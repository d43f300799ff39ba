#!/bin/bash
# Round 6: do the workgroups of one C2 launch alias in the memory system because they run in phase?  (1) row pitches
# whose contract stride (16 x pitch x 4 B) is an odd multiple of 4 KiB (pitch = odd x 64 floats) against the default
# 66,560; (2) a variant whose workgroups start staggered (tools/micro/v/libsmc_stagger.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/r06_desync_probe.txt
: > $out
for rep in 1 2; do
  for p in 66560 66624 66752 67648 65600; do
    echo -n "[pitch $p] " >> $out
    timeout -k 10 120 python tools/kprof_step.py --config c2 --iters 20 --pitch $p 2>/dev/null | grep -v amdgpu.ids >> $out || exit 1
  done
  echo -n "[stagger] " >> $out
  SMC_LIB_PATH=tools/micro/v/libsmc_stagger.so timeout -k 10 120 python tools/kprof_step.py --config c2 --iters 20 2>/dev/null | grep -v amdgpu.ids >> $out || exit 1
done
cat $out
