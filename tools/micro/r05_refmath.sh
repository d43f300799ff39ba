#!/bin/bash
# SMC_MATH_REF: the exchange-fault tests through the gated hook and the reference-math GPU tests, a C2 bench
# line in reference math (no CPU leg), then the f64 v4/v3 PMC passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-refmath}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_reference_math.py tests/test_gpu_engine.py tests/test_gpu_basket.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider -rf -k "reference_math or timeout" > $O/gputests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config c2 --math reference --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c2ref.out 2> $O/bench_c2ref.err || exit $?
bash tools/micro/r05_f64pmc.sh f64pmc
