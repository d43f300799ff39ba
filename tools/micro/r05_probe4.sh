#!/bin/bash
# round 5, GPU call 4: persistent fb_kernel with staged parameters / weights: GPU tests, then the narrow
# networks' step time (tools/kprof_net.py) for the new library (default), the previous one (fbold) and the
# previous one with 512-thread fb workgroups (fb512)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05p4; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_cvnn_mfma.py tests/test_gpu_trainer.py tests/test_gpu_reference_fixtures.py tests/test_gpu_c2_session.py tests/test_gpu_dp.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -rf > $O/tests.log 2>&1 || exit $?
for rep in 1 2; do
  for lib in default fbold fb512; do
    if [ $lib = default ]; then L=spectralmc_amd/libspectralmc_hip.so; else L=tools/micro/v/libsmc_$lib.so; fi
    for arch in lockstep e2e c2; do
      for opt in "--cus 32 --storm" "--cus 128 --storm" "--cus 0"; do
        echo -n "$lib: " >> $O/net_ab.txt
        SMC_LIB_PATH=$L timeout -k 10 120 python tools/kprof_net.py --arch $arch $opt 2>/dev/null | grep -v amdgpu.ids >> $O/net_ab.txt || exit $?
      done
    done
  done
done
