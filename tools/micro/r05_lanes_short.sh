#!/bin/bash
# e2e: MC lanes for short launches (pricer.mc_lanes_short) with the eager short steps, two passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-lanesshort}; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2; do
  for n in 1 2; do
    for cfg in e2e; do
      echo -n "$cfg lanes_short=$n: " >> $O/bench.txt
      timeout -k 10 300 python bench.py --config $cfg --steps 200 --warmup 5 --no-cpu-baseline --lanes-short $n 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['ms_per_step'],4), 'host', round(d['host_enqueue_ms_per_step'],4), 'kernel', round(r['kernel_ms'],4), 'live', r.get('kernel_ms_live'), 'steady', r.get('kernel_ms_steady'))" >> $O/bench.txt || exit $?
    done
  done
done
