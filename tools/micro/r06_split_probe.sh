#!/bin/bash
# Round 6: one C2 call (4096 contracts) as 1 launch on the whole chip vs 2 / 4 concurrent launches on complementary
# CU-masked streams (each with CUs of every XCD), static-quarter and dynamic contract queues; 2 passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r06_split_probe.txt; : > $o
for rep in 1 2; do
  for args in "" "--split 2" "--split 4" "--dynamic" "--dynamic --split 2" "--dynamic --split 4"; do
    echo -n "[$args] " >> $o
    timeout -k 10 120 python tools/kprof_step.py --config c2 --iters 10 $args 2>&1 | grep -v amdgpu.ids >> $o || exit 1
  done
done
cat $o
