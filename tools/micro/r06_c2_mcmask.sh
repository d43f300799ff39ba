#!/bin/bash
# Round 6: C2 step with the path lanes on the 224 CUs the network's mask leaves (default) vs on the whole chip
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r06_c2_mcmask.txt; : > $o
for rep in 1 2; do
  for m in on off; do
    echo -n "mc-cu-mask=$m: " >> $o
    timeout -k 10 300 python bench.py --steps 40 --warmup 5 --kernel-iters 2 --no-cpu-baseline --mc-cu-mask $m 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(f\"{d['ms_per_step']:.4f} ms/step, steady {r['kernel_ms_steady']}\")" >> $o || exit 1
  done
done
cat $o
