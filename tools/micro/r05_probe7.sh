#!/bin/bash
# round 5, GPU call 7: the fused Adam finalize with sc1 hand-off (default) vs round 4's library (r4: separate
# finalize launch, round-4 fb / lgemm): tests, the networks alone / beside a write storm, bench steps
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05p7; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_cvnn_mfma.py tests/test_gpu_trainer.py tests/test_gpu_dp.py tests/test_gpu_c2_session.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > $O/tests.log 2>&1 || exit $?
for rep in 1 2; do
  for lib in default r4; do
    if [ $lib = default ]; then L=spectralmc_amd/libspectralmc_hip.so; else L=tools/micro/v/libsmc_$lib.so; fi
    for spec in "h256:--cus 0" "h256:--cus 64 --storm" "c2:--cus 0" "c2:--cus 32 --storm" "lockstep:--cus 0" "lockstep:--cus 32 --storm" "e2e:--cus 0" "e2e:--cus 128 --storm"; do
      arch=${spec%%:*}; opt=${spec#*:}
      echo -n "$lib: " >> $O/net.txt
      SMC_LIB_PATH=$L timeout -k 10 120 python tools/kprof_net.py --arch $arch $opt 2>/dev/null | grep -v amdgpu.ids >> $O/net.txt || exit $?
    done
    for cfg in c2h256 c2 e2e; do
      echo -n "$lib $cfg: " >> $O/bench.txt
      SMC_LIB_PATH=$L timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 3 --kernel-iters 2 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), 'kernel', round(d['roofline']['kernel_ms'],4), 'net', round(d['network']['ms'],4))" >> $O/bench.txt || exit $?
    done
    echo -n "$lib lockstep: " >> $O/bench.txt
    [ $lib = default ] && { SMC_LIB_PATH=$L timeout -k 10 200 python bench.py --config lockstep --steps 40 --warmup 3 --kernel-iters 2 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), 'kernel', round(d['roofline']['kernel_ms'],4), 'net', round(d['network']['ms'],4))" >> $O/bench.txt || exit $?; } || echo "(r4 library: RAW query flag of ABI 11)" >> $O/bench.txt
  done
done
