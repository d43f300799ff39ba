#!/bin/bash
# Round 6: four MC lanes with smaller launches (B = 1024 / 2048 per launch): per-contract rate of launches in flight
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r06_lanes_small.txt; : > $o
for rep in 1 2; do
  for args in "--lanes 4 --B 4096 --iters 16" "--lanes 4 --B 2048 --iters 32" "--lanes 4 --B 1024 --iters 64" "--B 4096 --iters 16"; do
    echo -n "[$args] " >> $o
    timeout -k 10 120 python tools/kprof_step.py --config c2 --dynamic $args 2>/dev/null | grep -v amdgpu.ids >> $o || exit 1
  done
done
sed -E 's/c2 normalize pitch=66560 (B=[0-9]+).*resident_kernel: ([0-9.]+ ms\/step).*/\1 \2/' $o
