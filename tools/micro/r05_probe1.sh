#!/bin/bash
# round 5, GPU call: C2 store-order probes (storebench8), sliced-C2 variants, isolated rocprof of the MC launch
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05p1; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 120 tools/micro/v/storebench8 > $O/storebench8.txt 2>&1 || exit $?
bash tools/micro/ab.sh $O/ab_sliced_c2.txt "--config c2 --iters 10" default ws2 ws4 default || exit $?
