#!/bin/bash
# C2/H=256 bench lines (no CPU leg), default library (kLM = 64) vs tools/micro/libsmc_m128.so, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/h256_ab.txt; : > $out
for round in 1 2; do
  timeout -k 10 300 python3 bench.py --config c2h256 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/h256_m64.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/h256_m64.json').read().strip().split('\n')[-1]);print('m64', d['ms_per_step'], d['network']['ms'])" >> $out
  SMC_LIB_PATH=$PWD/tools/micro/libsmc_m128.so timeout -k 10 300 python3 bench.py --config c2h256 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/h256_m128.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/h256_m128.json').read().strip().split('\n')[-1]);print('m128', d['ms_per_step'], d['network']['ms'])" >> $out
done
cat $out
