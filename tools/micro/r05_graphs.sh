#!/bin/bash
# short shapes: captured step graphs (default) against eager launches (--graphs off), two passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-graphs}; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2; do
for cfg in e2e lockstep; do
  for g in on off; do
    echo -n "$cfg graphs=$g: " >> $O/bench.txt
    timeout -k 10 300 python bench.py --config $cfg --steps 200 --warmup 5 --no-cpu-baseline --graphs $g 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['ms_per_step'],4), 'host', round(d['host_enqueue_ms_per_step'],4), 'kernel', round(d['roofline']['kernel_ms'],4))" >> $O/bench.txt || exit $?
  done
done
done
