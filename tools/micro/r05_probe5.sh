#!/bin/bash
# round 5, GPU call 5: bench lock-step / e2e / C2 step times with the persistent fb_kernel (default), its 512-thread
# form (fbp512), the round-4 fb_kernel (fbold) and that at 512 threads (fb512)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05p5; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2; do
  for lib in default fbp512 fbold fb512; do
    if [ $lib = default ]; then L=spectralmc_amd/libspectralmc_hip.so; else L=tools/micro/v/libsmc_$lib.so; fi
    for cfg in lockstep e2e; do
      echo -n "$lib $cfg: " >> $O/bench_ab.txt
      SMC_LIB_PATH=$L timeout -k 10 200 python bench.py --config $cfg --steps 40 --warmup 3 --kernel-iters 2 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), 'kernel', round(d['roofline']['kernel_ms'],4), 'net', round(d['network']['ms'],4))" >> $O/bench_ab.txt || exit $?
    done
  done
done
