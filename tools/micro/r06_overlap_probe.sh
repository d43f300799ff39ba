#!/bin/bash
# Round 6: why do overlapped C2 launches (MC lanes) run faster per contract than one launch alone?  The same
# smc_train_step launches one at a time (static / dynamic contract assignment), with 2 and 4 lanes, and as one
# launch of twice the contracts; C3's launch alone for comparison.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=gpurun_out/r06_overlap_probe.txt
: > $out
for rep in 1 2; do
  for args in "--config c2 --iters 20" "--config c2 --iters 20 --dynamic" "--config c2 --iters 20 --lanes 2 --dynamic" \
              "--config c2 --iters 20 --lanes 4 --dynamic" "--config c2 --iters 10 --B 8192" "--config c2 --iters 10 --B 16384"; do
    echo -n "[$args] " >> $out
    timeout -k 10 120 python tools/kprof_step.py $args 2>/dev/null | grep -v amdgpu.ids >> $out || exit 1
  done
done
timeout -k 10 200 python tools/kprof_step.py --config c3 --iters 2 2>/dev/null | grep -v amdgpu.ids >> $out || exit 1
cat $out
