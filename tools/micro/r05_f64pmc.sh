#!/bin/bash
# f64 math v4 vs v3 under PMC: clock / VALU issue (GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES) and LDS
# (SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE) of the C2-f64 launches, one rocprofv3 pass per counter set
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$PWD; O=gpurun_out/${1:-f64pmc}; mkdir -p $O; export TMPDIR=/tmp
for lib in v4 v3; do
  if [ $lib = v4 ]; then export SMC_LIB_PATH=$ROOT/spectralmc_amd/libspectralmc_hip.so; else export SMC_LIB_PATH=$ROOT/tools/micro/v/libsmc_f64v3.so; fi
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv \
    -d $O/clock_$lib -o run -- python3 $ROOT/tools/kprof_step.py --config c2 --dtype f64 --iters 4 > $O/clock_$lib.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv \
    -d $O/lds_$lib -o run -- python3 $ROOT/tools/kprof_step.py --config c2 --dtype f64 --iters 4 > $O/lds_$lib.log 2>&1 || exit $?
done
