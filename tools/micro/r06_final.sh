#!/bin/bash
# Round-6 closing measurements -> gpurun_out/final6 (tools/r06_records.py copies them to profiles/r06/final): per
# config one bench line with the CPU baseline (c2 only: the default command), the rocprofv3 kernel stats + trace of
# the same command without the CPU leg (its last kernel_iters dispatches of the dominant kernel are the launches the
# line's kernel_ms times), and the rocprofv3 stats of the dominant launch alone (tools/kprof_step.py /
# kprof_basket.py); PMC passes (traffic, clock / VALU) over the C2, C2-f64 and reference-math launches.
#   tools/micro/r06_final.sh c2 c2h256 c3 c5 lockstep e2e c2f64 c2ref c2refhw pmc
set -u
cd "${GRAFT_REPO_ROOT:-.}"
ROOT=$(pwd)
export TMPDIR=/tmp
O=$ROOT/gpurun_out/final6
mkdir -p $O
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[$(date +%T)] $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.out" 2> "$O/$name.err" || { echo "FAILED $name rc=$?"; tail -5 "$O/$name.err"; exit 1; }
}
pmc() {  # tag kprof-args counters...
  local tag=$1 args=$2; shift 2
  cd /tmp
  step pmc_$tag 180 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $O/pmc_$tag -o run -- python3 $ROOT/tools/kprof_step.py $args
  cd $ROOT
}
for cfg in "$@"; do
  if [ "$cfg" = pmc ]; then
    for ctr in WRITE_SIZE FETCH_SIZE; do pmc c2_$ctr "--config c2 --dynamic --iters 3" $ctr; done
    pmc c2_clock "--config c2 --dynamic --iters 3" GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES
    pmc c2f64_clock "--config c2 --dtype f64 --iters 3" GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES
    for ctr in WRITE_SIZE FETCH_SIZE; do pmc c2ref_$ctr "--config c2 --math reference --iters 3" $ctr; done
    pmc c2ref_clock "--config c2 --math reference --iters 3" GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU
    pmc c2ref_lds "--config c2 --math reference --iters 3" SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES
    pmc c2refhw_clock "--config c2 --math reference_hw --iters 3" GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU
    continue
  fi
  steps=20; warm=3; args="--config $cfg"
  case "$cfg" in c3|c5) steps=5; warm=2 ;; c2f64) steps=10 ;; c2ref) steps=10; args="--config c2 --math reference" ;; c2refhw) steps=10; args="--config c2 --math reference_hw" ;; esac
  if [ "$cfg" = c2 ]; then step bench_c2 420 python bench.py; else step bench_$cfg 420 python bench.py $args --steps $steps --warmup $warm --no-cpu-baseline; fi
  cd /tmp
  step prof_$cfg 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$cfg -o run -- python3 $ROOT/bench.py $args --no-cpu-baseline --steps $steps --warmup $warm
  case "$cfg" in
    c2|c2h256) drv="$ROOT/tools/kprof_step.py --config c2 --dynamic --iters 10" ;;
    c3) drv="$ROOT/tools/kprof_step.py --config c3 --iters 4" ;;
    c5) chunk=$(python3 -c "import json;print(json.loads(open('$O/bench_c5.out').read().strip().splitlines()[-1])['roofline']['contracts_per_launch'])"); drv="$ROOT/tools/kprof_basket.py --B $chunk --iters 4" ;;
    lockstep|e2e) drv="$ROOT/tools/kprof_step.py --config $cfg --dynamic --iters 20" ;;
    c2f64) drv="$ROOT/tools/kprof_step.py --config c2 --dtype f64 --iters 4" ;;
    c2ref) drv="$ROOT/tools/kprof_step.py --config c2 --math reference --iters 4" ;;
    c2refhw) drv="$ROOT/tools/kprof_step.py --config c2 --math reference_hw --iters 4" ;;
  esac
  step iso_$cfg 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/iso_$cfg -o run -- python3 $drv
  cd $ROOT
done
echo done
