#!/bin/bash
# Round 6: C2-f64 step with the f64 network beside the next rows launch (default) vs sequential, two passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
o=gpurun_out/r06_f64_overlap.txt; : > $o
for rep in 1 2; do
  for ov in on off; do
    echo -n "overlap-rows=$ov: " >> $o
    timeout -k 10 300 python bench.py --config c2f64 --steps 10 --warmup 3 --kernel-iters 2 --no-cpu-baseline --overlap-rows $ov 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(f\"{d['ms_per_step']:.3f} ms/step, kernel {r['kernel_ms']:.3f}, live {r.get('kernel_ms_live')}, net {d['network']['ms']:.3f}\")" >> $o || exit 1
  done
done
cat $o
