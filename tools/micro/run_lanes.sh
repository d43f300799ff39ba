#!/bin/bash
# C2 MC part on 1 stream vs launches alternating over 2 streams (tools/kprof_step.py --lanes), with the
# default static contract share or every contract from the queue (--dynamic).
set -u
out=$1; shift
for rep in 1 2; do
  for args in "--lanes 1" "--lanes 1 --dynamic" "--lanes 2" "--lanes 2 --dynamic"; do
    echo -n "$args: " >> "$out"
    timeout -k 10 120 python tools/kprof_step.py --config c2 --iters 20 $args 2>/dev/null | grep -v amdgpu.ids >> "$out" || exit 1
  done
done
