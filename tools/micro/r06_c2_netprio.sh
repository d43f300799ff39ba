#!/bin/bash
# Round 6: C2 step with an unmasked network at each stream priority against the default (32 masked CUs)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r06_c2_netprio.txt; : > $o
for rep in 1 2; do
  for cfg in "--net-cus 32" "--net-cus 0 --priority none" "--net-cus 0 --priority mc" "--net-cus 0 --priority network"; do
    echo -n "[$cfg] " >> $o
    timeout -k 10 300 python bench.py --steps 40 --warmup 5 --kernel-iters 2 --no-cpu-baseline $cfg 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(f\"{d['ms_per_step']:.4f} ms/step, steady {r['kernel_ms_steady']}\")" >> $o || exit 1
  done
done
cat $o
