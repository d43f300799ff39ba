#!/bin/bash
# C2-f64: the f64 network beside the next rows launch (pricer.overlap_rows on) or after it (off), two passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-f64overlap}; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2; do
  for o in on off; do
    echo -n "c2f64 overlap_rows=$o: " >> $O/bench.txt
    timeout -k 10 300 python bench.py --config c2f64 --steps 12 --warmup 3 --no-cpu-baseline --kernel-iters 2 --overlap-rows $o 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['ms_per_step'],4), 'kernel', round(r['kernel_ms'],4), 'live', r.get('kernel_ms_live'))" >> $O/bench.txt || exit $?
  done
done
