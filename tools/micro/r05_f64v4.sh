#!/bin/bash
# f64 math v4: the GPU tests that run f64 paths, then an interleaved A/B of the C2-f64 step (v4 in-tree vs the
# v3 library libsmc_f64v3.so) and the c2f64 bench line (no CPU leg)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-f64v4}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_reference_fixtures.py tests/test_gpu_trainer.py \
  -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -rf -k "f64 or float64 or normals or lockstep" > $O/gputests.log 2>&1 || exit $?
tools/micro/ab.sh $O/ab_c2f64.txt "--config c2 --dtype f64" default f64v3 || exit $?
timeout -k 10 300 python bench.py --config c2f64 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c2f64.out 2> $O/bench_c2f64.err || exit $?
