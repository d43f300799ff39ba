#!/bin/bash
# host enqueue time against the step time at the short shapes (bench lines without the CPU leg)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-host}; mkdir -p $O; export TMPDIR=/tmp
for cfg in e2e lockstep c2; do
  timeout -k 10 300 python bench.py --config $cfg --steps 200 --warmup 5 --no-cpu-baseline > $O/bench_$cfg.out 2> $O/bench_$cfg.err || exit $?
done
