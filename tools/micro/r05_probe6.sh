#!/bin/bash
# round 5, GPU call 6: lgemm_kernel with two register sets of staged loads (default) vs round 4's (lgold): MFMA
# tests, the H = 256 network alone / on 64 masked CUs beside a write storm, and the C2/H=256 bench step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05p6; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_cvnn_mfma.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -rf > $O/tests.log 2>&1 || exit $?
for rep in 1 2; do
  for lib in default lgold; do
    if [ $lib = default ]; then L=spectralmc_amd/libspectralmc_hip.so; else L=tools/micro/v/libsmc_$lib.so; fi
    for opt in "--cus 0" "--cus 64 --storm"; do
      echo -n "$lib: " >> $O/net_h256.txt
      SMC_LIB_PATH=$L timeout -k 10 120 python tools/kprof_net.py --arch h256 $opt 2>/dev/null | grep -v amdgpu.ids >> $O/net_h256.txt || exit $?
    done
    echo -n "$lib c2h256: " >> $O/bench_h256.txt
    SMC_LIB_PATH=$L timeout -k 10 200 python bench.py --config c2h256 --steps 20 --warmup 3 --kernel-iters 2 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), 'kernel', round(d['roofline']['kernel_ms'],4), 'net', round(d['network']['ms'],4))" >> $O/bench_h256.txt || exit $?
  done
done
