#!/bin/bash
# bench.py A/B: each argument is one quoted set of bench.py flags; prints ms/step, the live MC-part
# time and their difference.  Usage: tools/micro/run_bench_ab.sh OUT.txt "--priority mc" "..."
set -u
out=$1; shift
for flags in "$@"; do
  line=$(timeout -k 10 200 python bench.py --steps 40 --warmup 4 --no-cpu-baseline $flags 2>/dev/null | tail -1) || exit 1
  python3 -c "import json,sys; d=json.loads(sys.argv[1]); r=d['roofline']; print(f\"{sys.argv[2]:28s} ms/step {d['ms_per_step']:.4f}  mc live {r['kernel_ms']:.4f}  gap {1e3*(d['ms_per_step']-r['kernel_ms']):.1f} us\")" "$line" "$flags" >> "$out"
done
