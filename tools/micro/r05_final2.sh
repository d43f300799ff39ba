#!/bin/bash
# Round-5 closing measurements -> gpurun_out/final5 (copied to profiles/r05): per config one bench line with the
# CPU baseline, the rocprofv3 kernel stats of the same command (no CPU leg), and the rocprofv3 stats of the
# dominant launch alone in the shape the bench's kernel_ms times (tools/kprof_step.py / kprof_basket.py);
# WRITE_SIZE / FETCH_SIZE and clock passes over the C2 launch.  Stops at the first failing step.
#   tools/micro/r05_final.sh c2 c2h256 c3 c5 lockstep e2e c2f64
set -u
cd "${GRAFT_REPO_ROOT:-.}"
ROOT=$(pwd)
export TMPDIR=/tmp
O=$ROOT/gpurun_out/${FINAL_DIR:-final5}
mkdir -p $O
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[$(date +%T)] $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.out" 2> "$O/$name.err" || { echo "FAILED $name rc=$?"; tail -5 "$O/$name.err"; exit 1; }
}
for cfg in "$@"; do
  steps=20; warm=3
  case "$cfg" in c3|c5) steps=5; warm=2 ;; c2f64) steps=10 ;; esac
  if [ "$cfg" = c2 ]; then step bench_c2 420 python bench.py; else step bench_$cfg 420 python bench.py --config $cfg --steps $steps --warmup $warm; fi
  cd /tmp
  step prof_$cfg 420 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$cfg -o run -- python3 $ROOT/bench.py --config $cfg --no-cpu-baseline --steps $steps --warmup $warm
  case "$cfg" in
    c2|c2h256) drv="$ROOT/tools/kprof_step.py --config c2 --dynamic --iters 10" ;;
    c3) drv="$ROOT/tools/kprof_step.py --config c3 --iters 4" ;;
    c5) chunk=$(python3 -c "import json;print(json.loads(open('$O/bench_c5.out').read().strip().splitlines()[-1])['roofline']['contracts_per_launch'])"); drv="$ROOT/tools/kprof_basket.py --B $chunk --iters 4" ;;
    lockstep|e2e) drv="$ROOT/tools/kprof_step.py --config $cfg --dynamic --iters 20" ;;
    c2f64) drv="$ROOT/tools/kprof_step.py --config c2 --dtype f64 --iters 4" ;;
  esac
  step iso_$cfg 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/iso_$cfg -o run -- python3 $drv
  cd $ROOT
done
cd /tmp
[ "${PMC:-1}" = 1 ] || { echo done; exit 0; }
for ctr in WRITE_SIZE FETCH_SIZE; do
  step pmc_c2_$ctr 180 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d $O/pmc_c2_$ctr -o run -- python3 $ROOT/tools/kprof_step.py --config c2 --dynamic --iters 3
done
step pmc_c2_clock 180 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv -d $O/pmc_c2_clock -o run -- python3 $ROOT/tools/kprof_step.py --config c2 --dynamic --iters 3
step pmc_c2f64_clock 180 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES --output-format csv -d $O/pmc_c2f64_clock -o run -- python3 $ROOT/tools/kprof_step.py --config c2 --dtype f64 --iters 3
echo done
