#!/bin/bash
# Round 6: C3 / C5 steps with the network on 32 CU-masked CUs beside the exchanging launch (--exchanging-masks on)
# against the default (the network after the launch, whole chip), two interleaved passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r06_xmasks.txt; : > $o
for rep in 1 2; do
  for cfg in c3 c5; do
    for m in off on; do
      echo -n "$cfg masks=$m: " >> $o
      timeout -k 10 300 python bench.py --config $cfg --steps 5 --warmup 2 --kernel-iters 1 --no-cpu-baseline --exchanging-masks $m 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(f\"{d['ms_per_step']:.3f} ms/step, kernel {r['kernel_ms']:.3f} ms, live {r.get('kernel_ms_live')}\")" >> $o || exit 1
    done
  done
done
cat $o
