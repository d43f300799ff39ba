#!/bin/bash
# eager short steps on explicit stream handles: the GPU suite, then bench lines (two passes)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-eager}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > $O/gputests.log 2>&1 || exit $?
for rep in 1 2; do
for cfg in e2e lockstep c2; do
  echo -n "$cfg: " >> $O/bench.txt
  timeout -k 10 300 python bench.py --config $cfg --steps 200 --warmup 5 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['ms_per_step'],4), 'host', round(d['host_enqueue_ms_per_step'],4), 'kernel', round(d['roofline']['kernel_ms'],4))" >> $O/bench.txt || exit $?
done
done
