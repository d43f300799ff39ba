#!/bin/bash
# the driver's default bench command (python bench.py: C2, 20 steps, 3 warm-up, CPU baseline), one line per box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-c2default}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python bench.py > $O/bench.out 2> $O/bench.err || exit $?
python -c "import json; d=json.loads(open('$O/bench.out').read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['ms_per_step'],4), 'kernel', round(r['kernel_ms'],4), 'frac', round(r['frac'],4), 'steady', r.get('kernel_ms_steady'))" > $O/summary.txt
