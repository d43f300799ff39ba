#!/bin/bash
# bench.py A/B of variant libraries (tools/micro/make_variant.py): r05_ab_bench.sh OUT "bench args" name ...
# ("default": the in-tree library), interleaved over two passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
out=$1; args=$2; shift 2
mkdir -p "$(dirname "$out")"; export TMPDIR=/tmp
for rep in 1 2; do
  for name in "$@"; do
    if [ "$name" = default ]; then lib=spectralmc_amd/libspectralmc_hip.so; else lib=tools/micro/v/libsmc_$name.so; fi
    echo -n "$name: " >> "$out"
    SMC_LIB_PATH=$lib timeout -k 10 300 python bench.py $args --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['ms_per_step'],4), 'host', round(d['host_enqueue_ms_per_step'],4), 'kernel', round(d['roofline']['kernel_ms'],4), 'net', round(d['network']['ms'],4) if d.get('network') else None)" >> "$out" || exit 1
  done
done
