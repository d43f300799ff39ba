#!/bin/bash
# Round 6: C5 launch size through the path budget: default (3 x 2731), 70 GiB (4 x 2048), 50 GiB (6 x 1366)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r06_c5_budget2.txt; : > $o
for rep in 1 2; do
  for gb in default 70 50; do
    echo -n "budget=$gb: " >> $o
    if [ $gb = default ]; then env_=""; else env_="SMC_PATH_BUFFER_GB=$gb"; fi
    env $env_ timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 2 --kernel-iters 1 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(f\"{d['ms_per_step']:.3f} ms/step, {r['contracts_per_launch']} per launch, kernel {r['kernel_ms']:.3f}\")" >> $o || exit 1
  done
done
cat $o
