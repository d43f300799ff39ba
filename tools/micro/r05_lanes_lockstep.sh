#!/bin/bash
# lock-step shape: MC lanes 2 vs 4, three passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-laneslock}; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2 3; do
  for n in 2 4 1; do
    echo -n "lockstep lanes=$n: " >> $O/bench.txt
    timeout -k 10 300 python bench.py --config lockstep --steps 200 --warmup 5 --no-cpu-baseline --kernel-iters 2 --lanes $n 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['ms_per_step'],4), 'kernel', round(r['kernel_ms'],4), 'steady', r.get('kernel_ms_steady'))" >> $O/bench.txt || exit $?
  done
done
