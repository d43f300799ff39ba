#!/bin/bash
# round 5, GPU call 8: network CUs for the short shapes with this round's network chain
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05p8; mkdir -p $O
run() {  # tag args...
  local tag=$1; shift
  echo -n "$tag: " >> $O/netcus.txt
  timeout -k 10 200 python bench.py --steps 40 --warmup 3 --kernel-iters 2 --no-cpu-baseline "$@" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],4), 'kernel', round(d['roofline']['kernel_ms'],4))" >> $O/netcus.txt || exit $?
}
for rep in 1 2; do
  for c in 32 64 96; do run "lockstep net_cus=$c" --config lockstep --net-cus $c || exit $?; done
  run "lockstep lanes=1" --config lockstep --lanes 1 || exit $?
  for c in 64 96 128 160; do run "e2e net_cus_small=$c" --config e2e --net-cus-small $c || exit $?; done
  run "e2e lanes=1" --config e2e --lanes 1 || exit $?
done
