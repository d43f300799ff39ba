#!/bin/bash
# Round 6 (run with the chunking of commit c19b222, since reverted): C5 with 2 launches of 4096 (default budget,
# no slot rounding) vs a 97-GiB budget (3 launches of 2731, the chunking kept): profiles/r06/r06_c5_budget_samebox.txt
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r06_c5_budget.txt; : > $o
python -c "import torch; print('total_memory', torch.cuda.get_device_properties(0).total_memory)" >> $o 2>/dev/null
for rep in 1 2; do
  for gb in default 97; do
    echo -n "budget=$gb: " >> $o
    if [ $gb = default ]; then env_=""; else env_="SMC_PATH_BUFFER_GB=$gb"; fi
    env $env_ timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 2 --kernel-iters 1 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(f\"{d['ms_per_step']:.3f} ms/step, {r['contracts_per_launch']} per launch, kernel {r['kernel_ms']:.3f}\")" >> $o || exit 1
  done
done
cat $o
