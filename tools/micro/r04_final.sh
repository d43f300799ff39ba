#!/bin/bash
# Round-4 closing measurements: one bench line per config (with the CPU baseline), the rocprofv3 kernel
# stats of the same command, and separate WRITE_SIZE / FETCH_SIZE passes over the config's path launch
# (tools/kprof_step.py, or tools/kprof_basket.py for C5) -> gpurun_out/final4, copied to profiles/r04.
# Each step under its own time limit; the script stops at the first failure.
#   tools/micro/r04_final.sh c2 lockstep c2f64 ...      (configs of bench.py)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/final4
mkdir -p $O
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[$(date +%T)] $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.out" 2> "$O/$name.err" || { echo "FAILED $name rc=$?"; tail -5 "$O/$name.err"; exit 1; }
}
for cfg in "$@"; do
  steps=20
  [ "$cfg" = c3 ] || [ "$cfg" = c5 ] && steps=5
  step bench_$cfg 420 python bench.py --config $cfg --steps $steps
  step prof_$cfg 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$cfg -- python3 bench.py --config $cfg --no-cpu-baseline --steps $steps
  case "$cfg" in
    c5) drv="tools/kprof_basket.py" ;;
    c2h256) drv="tools/kprof_step.py --config c2 --iters 5" ;;
    c2f64) drv="tools/kprof_step.py --config c2 --dtype f64 --iters 3" ;;
    *) drv="tools/kprof_step.py --config $cfg --iters 5" ;;
  esac
  for ctr in WRITE_SIZE FETCH_SIZE; do
    step pmc_${cfg}_$ctr 180 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d $O/pmc_${cfg}_$ctr -- python3 $drv
  done
done
# the C2 path launch alone (one stream, full chip): the per-launch duration bench.py's roofline uses
step prof_isolated_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_isolated_c2 -- python3 tools/kprof_step.py --config c2 --iters 20
echo done
