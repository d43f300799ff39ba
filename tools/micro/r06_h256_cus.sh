#!/bin/bash
# Round 6: C2/H=256 step with the wide network on 32 / 64 / 96 masked CUs, beside C2 on the same box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r06_h256_cus.txt; : > $o
for rep in 1 2; do
  for cfg in "--config c2" "--config c2h256 --net-cus-wide 32" "--config c2h256 --net-cus-wide 64" "--config c2h256 --net-cus-wide 96"; do
    echo -n "[$cfg] " >> $o
    timeout -k 10 300 python bench.py --steps 40 --warmup 5 --kernel-iters 2 --no-cpu-baseline $cfg 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(f\"{d['ms_per_step']:.4f} ms/step, steady {r['kernel_ms_steady']}, net alone {d['network']['ms']:.4f}\")" >> $o || exit 1
  done
done
cat $o
