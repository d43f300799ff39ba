#!/bin/bash
# C2/H=256: CUs reserved for the wide network (pricer.network_cus_wide), interleaved over two passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-widecus}; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2; do
  for n in 64 32 96; do
    echo -n "c2h256 net_cus_wide=$n: " >> $O/bench.txt
    timeout -k 10 300 python bench.py --config c2h256 --steps 30 --warmup 3 --no-cpu-baseline --kernel-iters 2 --net-cus-wide $n 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['ms_per_step'],4), 'kernel', round(d['roofline']['kernel_ms'],4), 'net', round(d['network']['ms'],4))" >> $O/bench.txt || exit $?
  done
done
