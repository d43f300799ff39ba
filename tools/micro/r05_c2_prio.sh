#!/bin/bash
# C2 with four MC lanes: stream priority network (default) / none, three passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-c2prio}; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2 3; do
  for p in network none; do
    echo -n "c2 priority=$p: " >> $O/bench.txt
    timeout -k 10 300 python bench.py --config c2 --steps 40 --warmup 4 --no-cpu-baseline --kernel-iters 2 --priority $p 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['ms_per_step'],4), 'steady', r.get('kernel_ms_steady'))" >> $O/bench.txt || exit $?
  done
done
