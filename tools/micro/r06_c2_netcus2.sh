#!/bin/bash
# Round 6: C2 step with the network on 8 / 16 / 32 masked CUs (one, two or four per XCD), two passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r06_c2_netcus2.txt; : > $o
for rep in 1 2; do
  for n in 32 16 8; do
    echo -n "net-cus=$n: " >> $o
    timeout -k 10 300 python bench.py --steps 40 --warmup 5 --kernel-iters 2 --no-cpu-baseline --net-cus $n 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(f\"{d['ms_per_step']:.4f} ms/step, steady {r['kernel_ms_steady']}, net alone {d['network']['ms']:.4f}\")" >> $o || exit 1
  done
done
cat $o
