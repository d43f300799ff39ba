#!/bin/bash
# round 5, GPU call 3: the narrow networks' step alone / on masked CUs / beside an HBM write storm
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05p3; mkdir -p $O; export TMPDIR=/tmp
for arch in lockstep e2e c2; do
  for cus in 0 32 128; do
    for storm in "" "--storm"; do
      timeout -k 10 120 python tools/kprof_net.py --arch $arch --cus $cus $storm 2>/dev/null | grep -v amdgpu.ids >> $O/net_contention.txt || exit $?
    done
  done
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_ls32 -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/kprof_net.py --arch lockstep --cus 32 --storm > $GRAFT_REPO_ROOT/$O/prof_ls32.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_ls32q -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/kprof_net.py --arch lockstep --cus 32 > $GRAFT_REPO_ROOT/$O/prof_ls32q.log 2>&1 || exit $?
