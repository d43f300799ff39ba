#!/bin/bash
# Round-3 closing measurements: one bench line per config and the rocprofv3 kernel stats of the same
# command (profiles/r03/).  Each step under its own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[$(date +%T)] $name"
  timeout -k 10 "$lim" "$@" > "$O/$name.out" 2> "$O/$name.err" || { echo "FAILED $name rc=$?"; tail -5 "$O/$name.err"; exit 1; }
}
for cfg in "$@"; do
  extra=""
  [ "$cfg" != c2 ] && extra="--no-cpu-baseline"
  [ "$cfg" = c5 ] || [ "$cfg" = c3 ] && extra=""
  step bench_$cfg 300 python bench.py --config $cfg $extra
  step prof_$cfg 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$cfg -- python3 bench.py --config $cfg --no-cpu-baseline --steps 10
done
# the C2 path launch alone (one stream, full chip): the per-launch duration bench.py's roofline uses
step prof_isolated 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_isolated -- python3 tools/kprof_step.py --config c2 --iters 20
echo done
