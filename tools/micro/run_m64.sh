#!/bin/bash
# lgemm feature-tile A/B: the default library vs tools/micro/libsmc_m64.so (kLM = 64: twice the
# workgroups at H = 256) on the isolated H = 256 network step, then the MFMA parity tests on the variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python3 tools/kprof_net.py --arch h256 --compute mfma > gpurun_out/m64_base.txt 2>&1 || exit $?
SMC_LIB_PATH=$PWD/tools/micro/libsmc_m64.so timeout -k 10 120 python3 tools/kprof_net.py --arch h256 --compute mfma > gpurun_out/m64_var.txt 2>&1 || exit $?
timeout -k 10 120 python3 tools/kprof_net.py --arch h256 --compute mfma >> gpurun_out/m64_base.txt 2>&1 || exit $?
SMC_LIB_PATH=$PWD/tools/micro/libsmc_m64.so timeout -k 10 120 python3 tools/kprof_net.py --arch h256 --compute mfma >> gpurun_out/m64_var.txt 2>&1 || exit $?
grep us/step gpurun_out/m64_base.txt gpurun_out/m64_var.txt
SMC_LIB_PATH=$PWD/tools/micro/libsmc_m64.so timeout -k 10 300 python3 -m pytest tests/test_gpu_cvnn_mfma.py -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/m64_tests.txt 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/m64_tests.txt
