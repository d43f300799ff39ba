#!/bin/bash
# Round 6: split tail of the whole-contract resident launch -- parity on the GPU, then A/B of the C2 launch alone
# (one stream) and with four lanes, over tail variants (tools/micro/make_variant.py; old = the round-5 sources).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_c2_session.py tests/test_gpu_reference_fixtures.py \
  -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -rf > $OUT/r06_tail_tests.log 2>&1
rc=$?; tail -3 $OUT/r06_tail_tests.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 600 bash tools/micro/ab.sh $OUT/r06_ab_tail_iso.txt "--config c2 --iters 10" old default t0 t64s4 t128s8 t256s8 || exit $?
timeout -k 10 600 bash tools/micro/ab.sh $OUT/r06_ab_tail_lanes4.txt "--config c2 --iters 20 --lanes 4 --dynamic" old default t128s8 || exit $?
SMC_LIB_PATH=tools/micro/v/libsmc_trace.so timeout -k 10 120 python tools/kprof_step.py --config c2 --iters 5 --trace $OUT/trace_c2_tail.npy > $OUT/r06_trace_tail.txt 2>&1
cat $OUT/r06_ab_tail_iso.txt $OUT/r06_ab_tail_lanes4.txt $OUT/r06_trace_tail.txt
