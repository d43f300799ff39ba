#!/bin/bash
# e2e (eager short steps): stream priority network / mc / none, two passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-prioe2e}; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2; do
  for p in network mc none; do
    echo -n "e2e priority=$p: " >> $O/bench.txt
    timeout -k 10 300 python bench.py --config e2e --steps 200 --warmup 5 --no-cpu-baseline --priority $p 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['ms_per_step'],4), 'live', r.get('kernel_ms_live'))" >> $O/bench.txt || exit $?
  done
done
