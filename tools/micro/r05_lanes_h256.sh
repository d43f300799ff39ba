#!/bin/bash
# C2/H=256: MC lanes (pricer.mc_lanes 2 vs 4) beside the wide network, three passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-lanesh256}; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2 3; do
  for n in 2 4; do
    echo -n "c2h256 lanes=$n: " >> $O/bench.txt
    timeout -k 10 300 python bench.py --config c2h256 --steps 40 --warmup 4 --no-cpu-baseline --kernel-iters 2 --lanes $n 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['ms_per_step'],4), 'kernel', round(r['kernel_ms'],4), 'steady', r.get('kernel_ms_steady'))" >> $O/bench.txt || exit $?
  done
done
