#!/bin/bash
# the exchange-fault GPU tests through the environment-gated hook, then the f64 v4/v3 PMC passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-hooks}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_basket.py tests/test_gpu_exchange_safety.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider -rf -k "timeout or fault or exchange" > $O/gputests.log 2>&1 || exit $?
bash tools/micro/r05_f64pmc.sh f64pmc
