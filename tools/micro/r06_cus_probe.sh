#!/bin/bash
# Round 6: one C2 launch at a time on a CU-masked stream of N CUs (N / 32 per shader engine), and four lanes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r06_cus_probe.txt; : > $o
for rep in 1 2; do
  for n in 0 224 192 160 128; do
    for ln in 1 4; do
      echo -n "[cus=$n lanes=$ln] " >> $o
      timeout -k 10 120 python tools/kprof_step.py --config c2 --iters 16 --dynamic --cus $n --lanes $ln 2>/dev/null | grep -v amdgpu.ids >> $o || exit 1
    done
  done
done
sed -E 's/c2 normalize pitch=66560 (B=[0-9]+).*resident_kernel: ([0-9.]+ ms\/step).*/\1 \2/' $o
