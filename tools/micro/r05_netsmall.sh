#!/bin/bash
# e2e: CUs of the network beside short launches (pricer.network_cus_small), two passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-netsmall}; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2; do
  for n in 128 96 64 160; do
    echo -n "e2e net_cus_small=$n: " >> $O/bench.txt
    timeout -k 10 300 python bench.py --config e2e --steps 200 --warmup 5 --no-cpu-baseline --net-cus-small $n 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['ms_per_step'],4), 'host', round(d['host_enqueue_ms_per_step'],4), 'kernel', round(d['roofline']['kernel_ms'],4), 'live', d['roofline'].get('kernel_ms_live'))" >> $O/bench.txt || exit $?
  done
done
