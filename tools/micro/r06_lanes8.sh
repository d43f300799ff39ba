#!/bin/bash
# Round 6: C2 path launches in flight: 4 vs 6 vs 8 lanes (kprof, no network), on all CUs and on 224
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r06_lanes8.txt; : > $o
for rep in 1 2; do
  for ln in 4 6 8; do
    for c in 0 224; do
      echo -n "[lanes=$ln cus=$c] " >> $o
      timeout -k 10 120 python tools/kprof_step.py --config c2 --iters 24 --dynamic --lanes $ln --cus $c 2>/dev/null | grep -v amdgpu.ids >> $o || exit 1
    done
  done
done
sed -E 's/c2 normalize pitch=66560 (B=[0-9]+).*resident_kernel: ([0-9.]+ ms\/step).*/\1 \2/' $o
