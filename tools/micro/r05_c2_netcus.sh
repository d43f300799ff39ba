#!/bin/bash
# C2 with four MC lanes: network CUs (pricer.network_cus) 32 vs 64, three passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-c2netcus}; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2 3; do
  for n in 32 64; do
    echo -n "c2 net_cus=$n: " >> $O/bench.txt
    timeout -k 10 300 python bench.py --config c2 --steps 40 --warmup 4 --no-cpu-baseline --kernel-iters 2 --net-cus $n 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['ms_per_step'],4), 'kernel', round(r['kernel_ms'],4), 'steady', r.get('kernel_ms_steady'))" >> $O/bench.txt || exit $?
  done
done
