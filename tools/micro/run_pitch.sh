#!/bin/bash
# Row-pitch sweep of the C2 MC part (tools/kprof_step.py), pitches in elements.
# Usage: tools/micro/run_pitch.sh OUT.txt pitch [pitch ...]
set -u
out=$1; shift
for p in "$@"; do
  timeout -k 10 120 python tools/kprof_step.py --config c2 --iters 10 --pitch "$p" 2>/dev/null | grep -v amdgpu.ids >> "$out" || exit 1
done
