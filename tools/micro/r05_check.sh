#!/bin/bash
# GPU suite, then short bench lines (no CPU leg) of the configs whose network part changed
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-check}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > $O/gputests.log 2>&1 || exit $?
for cfg in c2 c2h256 e2e lockstep; do
  echo -n "$cfg: " >> $O/bench.txt
  timeout -k 10 200 python bench.py --config $cfg --steps 30 --warmup 3 --kernel-iters 2 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), 'kernel', round(d['roofline']['kernel_ms'],4), 'frac', round(d['roofline']['frac'],4), 'net', round(d['network']['ms'],4))" >> $O/bench.txt || exit $?
done
