#!/bin/bash
# rocprofv3 kernel stats of the H=256 network step (tools/kprof_net.py) per library variant
# ("default" = the in-tree library).  Usage: tools/micro/run_net_variants.sh name [name ...]
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for name in "$@"; do
  if [ "$name" = default ]; then lib=spectralmc_amd/libspectralmc_hip.so; else lib=tools/micro/libsmc_$name.so; fi
  SMC_LIB_PATH=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/net_$name -- python3 tools/kprof_net.py --arch h256 --iters 20 > gpurun_out/net_$name.log 2>&1 || exit 1
done
