#!/bin/bash
# cProfile of the e2e bench in eager mode (host-bound): where the host time of a step goes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/${1:-hostprof}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -m cProfile -o $O/e2e_eager.prof bench.py --config e2e --steps 400 --warmup 5 --no-cpu-baseline --graphs off --kernel-iters 2 > $O/bench.out 2> $O/bench.err || exit $?
python - <<'PY' > gpurun_out/${1:-hostprof}/stats.txt
import pstats, sys
st = pstats.Stats(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/hostprof/e2e_eager.prof")
st.sort_stats("tottime").print_stats(45)
PY
