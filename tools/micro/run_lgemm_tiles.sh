#!/bin/bash
# lgemm tile A/B on the isolated H = 256 network step: default vs tools/micro/libsmc_<v>.so for each
# named variant (alternating, two rounds), then the MFMA parity tests on each variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/lgemm_tiles.txt; : > $out
for round in 1 2; do
  timeout -k 10 120 python3 tools/kprof_net.py --arch h256 --compute mfma | sed "s/^/base /" >> $out 2>&1 || exit 1
  for v in "$@"; do
    SMC_LIB_PATH=$PWD/tools/micro/libsmc_$v.so timeout -k 10 120 python3 tools/kprof_net.py --arch h256 --compute mfma \
      | sed "s/^/$v /" >> $out 2>&1 || exit 1
  done
done
grep us/step $out
for v in "$@"; do
  SMC_LIB_PATH=$PWD/tools/micro/libsmc_$v.so timeout -k 10 300 python3 -m pytest tests/test_gpu_cvnn_mfma.py -q -x \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/tiles_tests_$v.txt 2>&1
  echo "$v tests rc=$?"
done
