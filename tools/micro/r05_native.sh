#!/bin/bash
# (historical: the --native-step option and smc_session_step were reverted after this measurement,
#  profiles/r05/ab_native_session_step.txt; the script no longer runs against the current tree)
# native steady-state step: trainer / session GPU tests, then bench lines with the native step on and off
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-native}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_trainer.py tests/test_gpu_c2_session.py tests/test_gpu_reference_math.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider -rf > $O/gputests.log 2>&1 || exit $?
for rep in 1 2; do
for cfg in e2e lockstep c2; do
  for nat in on off; do
    echo -n "$cfg native=$nat: " >> $O/bench.txt
    timeout -k 10 300 python bench.py --config $cfg --steps 200 --warmup 5 --no-cpu-baseline --native-step $nat 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['ms_per_step'],4), 'host', round(d['host_enqueue_ms_per_step'],4), 'kernel', round(d['roofline']['kernel_ms'],4))" >> $O/bench.txt || exit $?
  done
done
done
