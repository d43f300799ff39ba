#!/bin/bash
# GPU-box driver: runs named steps, each under its own time limit; stops the whole call at
# the first fault / abort / timeout (exit >= 124, 134, 139) but continues past ordinary test
# failures (exit 1).  Usage: tools/gpu_run.sh step1 step2 ...   (steps defined below)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp

run() {
  local name=$1 limit=$2; shift 2
  echo "[$(date +%T)] start $name"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc"
  tail -n 5 "$OUT/$name.log"
  if [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; then
    echo "fatal exit $rc in $name: stopping"
    exit "$rc"
  fi
}

for step in "$@"; do
  case "$step" in
    info)    run info 120 bash -c "rocm-smi --showproductname; nproc; python -c 'import torch;print(torch.__version__, torch.cuda.get_device_name(0))'" ;;
    engine)  run engine 900 python -m pytest tests/test_gpu_engine.py -q -rf ;;
    trainer) run trainer 900 python -m pytest tests/test_gpu_trainer.py -q -rf ;;
    gputests) run gputests 1200 python -m pytest tests -m gpu -q -rf ;;
    smoke)   run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)   run bench 600 python bench.py ;;
    bench_quick) run bench_quick 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --math portable ;;
    bench_hw) run bench_hw 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --math hw ;;
    bench_hw_terminal) run bench_hw_terminal 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --store terminal --math hw ;;
    bench_terminal) run bench_terminal 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --store terminal --math portable ;;
    bench_c1) run bench_c1 600 python bench.py --config c1 --steps 50 --warmup 5 --no-cpu-baseline ;;
    basket)  run basket 600 python -u -m pytest tests/test_gpu_basket.py -x -v --timeout 120 --timeout-method thread -rf ;;
    dp)      run dp 600 python -u -m pytest tests/test_gpu_dp.py -x -v --timeout 300 --timeout-method thread -rf ;;
    bench_c5) run bench_c5 600 python bench.py --config c5 --steps 10 --warmup 3 --kernel-iters 2 ;;
    prof_c5) cd /tmp && run prof_c5 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_c5" -o run --output-format csv -- python "$ROOT/bench.py" --config c5 --steps 5 --warmup 2 --kernel-iters 1 --no-cpu-baseline; cd "$ROOT" ;;
    bench_h256) run bench_h256 600 python bench.py --config c2h256 --steps 20 --warmup 3 --no-cpu-baseline ;;
    bench_seq) run bench_seq 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --overlap off ;;
    prof_seq) cd /tmp && run prof_seq 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_seq" -o run --output-format csv -- python "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --overlap off; cd "$ROOT" ;;
    bench_nograph) run bench_nograph 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --graphs off ;;
    bench_seq_nograph) run bench_seq_nograph 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --graphs off --overlap off ;;
    bench_q) run bench_q 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline ;;
    bench_valu) run bench_valu 600 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --network valu ;;
    bench_c3_f32) run bench_c3_f32 900 python bench.py --config c3 --steps 3 --warmup 2 --kernel-iters 1 --no-cpu-baseline --network mfma ;;
    gputests_v) run gputests_v 1100 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -p no:cacheprovider -rf ;;
    bench_c3) run bench_c3 900 python bench.py --config c3 --steps 3 --warmup 2 --kernel-iters 1 --no-cpu-baseline ;;
    prof)    cd /tmp && run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline; cd "$ROOT" ;;
    prof_default) cd /tmp && run prof_default 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof_default" -o run --output-format csv -- python "$ROOT/bench.py"; cd "$ROOT" ;;
    prof_hw) cd /tmp && run prof_hw 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_hw" -o run --output-format csv -- python "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --math hw; cd "$ROOT" ;;
    pmc_c5_sq) cd /tmp && run pmc_c5_sq 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE -d "$OUT/pmc_c5_sq" -o run --output-format csv -- python "$ROOT/tools/kprof_basket.py"; cd "$ROOT" ;;
    pmc_c5_write) cd /tmp && run pmc_c5_write 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_c5_write" -o run --output-format csv -- python "$ROOT/tools/kprof_basket.py"; cd "$ROOT" ;;
    pmc_c5_fetch) cd /tmp && run pmc_c5_fetch 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_c5_fetch" -o run --output-format csv -- python "$ROOT/tools/kprof_basket.py"; cd "$ROOT" ;;
    pmc_c3_write) cd /tmp && run pmc_c3_write 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_c3_write" -o run --output-format csv -- python "$ROOT/tools/kprof.py" --math hw --store all --unsliced --B 2048 --N 1024 --M 256 --iters 3; cd "$ROOT" ;;
    pmc_c3_fetch) cd /tmp && run pmc_c3_fetch 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_c3_fetch" -o run --output-format csv -- python "$ROOT/tools/kprof.py" --math hw --store all --unsliced --B 2048 --N 1024 --M 256 --iters 3; cd "$ROOT" ;;
    pmc_c2_write) cd /tmp && run pmc_c2_write 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_c2_write" -o run --output-format csv -- python "$ROOT/tools/kprof.py" --math hw --store all --unsliced; cd "$ROOT" ;;
    pmc_c2_fetch) cd /tmp && run pmc_c2_fetch 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_c2_fetch" -o run --output-format csv -- python "$ROOT/tools/kprof.py" --math hw --store all --unsliced; cd "$ROOT" ;;
    pmc_hw_all)  cd /tmp && run pmc_hw_all 600 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE -d "$OUT/pmc_hw_all" -o run --output-format csv -- python "$ROOT/tools/kprof.py" --math hw --store all --unsliced; cd "$ROOT" ;;
    pmc_hw_term) cd /tmp && run pmc_hw_term 600 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE -d "$OUT/pmc_hw_term" -o run --output-format csv -- python "$ROOT/tools/kprof.py" --math hw --store terminal --unsliced; cd "$ROOT" ;;
    pmc_hw_bytes) cd /tmp && run pmc_hw_bytes 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_hw_bytes" -o run --output-format csv -- python "$ROOT/tools/kprof.py" --math hw --store all --unsliced; cd "$ROOT" ;;
    pmc_hw_fetch) cd /tmp && run pmc_hw_fetch 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_hw_fetch" -o run --output-format csv -- python "$ROOT/tools/kprof.py" --math hw --store all --unsliced; cd "$ROOT" ;;
    orderbench) run orderbench 240 tools/micro/orderbench ;;
    prof_order) cd /tmp && run prof_order 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_order" -o run --output-format csv -- "$ROOT/tools/micro/orderbench"; cd "$ROOT" ;;
    valurate) run valurate 120 tools/micro/valurate ;;
    ab_resident) run ab_resident 900 bash tools/micro/ab_resident.sh ;;
    pmcstep:*)  # pmcstep:<config>:<counter>[:iters] -> rocprofv3 PMC pass over tools/kprof_step.py
      IFS=: read -r _ cfg ctr its <<< "$step"
      cd /tmp && run "pmc_${cfg}_${ctr}" 300 rocprofv3 --kernel-trace --pmc "$ctr" -d "$OUT/pmc_${cfg}_${ctr}" -o run --output-format csv -- python "$ROOT/tools/kprof_step.py" --config "$cfg" --iters "${its:-3}"; cd "$ROOT" ;;
    profbench:*)  # profbench:<config>[:steps] -> rocprofv3 kernel stats of bench.py (no CPU leg)
      IFS=: read -r _ cfg st <<< "$step"
      cd /tmp && run "prof_${cfg}" 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${cfg}" -o run --output-format csv -- python "$ROOT/bench.py" --config "$cfg" --steps "${st:-5}" --warmup 2 --kernel-iters 2 --no-cpu-baseline; cd "$ROOT" ;;
    profstep:*)  # profstep:<config>[:iters] -> rocprofv3 kernel stats of the MC launch alone (tools/kprof_step.py)
      IFS=: read -r _ cfg its <<< "$step"
      cd /tmp && run "profstep_${cfg}" 300 rocprofv3 --kernel-trace --stats -d "$OUT/profstep_${cfg}" -o run --output-format csv -- python "$ROOT/tools/kprof_step.py" --config "$cfg" --iters "${its:-10}"; cd "$ROOT" ;;
    benchcfg:*)  # benchcfg:<config>[:steps] -> bench.py line with the CPU baseline
      IFS=: read -r _ cfg st <<< "$step"
      run "bench_${cfg}" 900 python bench.py --config "$cfg" --steps "${st:-10}" --warmup 3 --kernel-iters 2 ;;
    kstep:*)  # kstep:<config>[:extra args with , for spaces]
      IFS=: read -r _ cfg extra <<< "$step"
      run "kstep_${cfg}" 300 python tools/kprof_step.py --config "$cfg" ${extra//,/ } ;;
    pmcf64:*)  # pmcf64:<counters with , for spaces> -> PMC pass over the f64 C2 MC launch
      IFS=: read -r _ ctrs <<< "$step"; tag=$(echo "$ctrs" | tr ',' '_' | cut -c1-40)
      cd /tmp && run "pmcf64_$tag" 300 rocprofv3 --kernel-trace --pmc ${ctrs//,/ } -d "$OUT/pmcf64_$tag" -o run --output-format csv -- python "$ROOT/tools/kprof_step.py" --config c2 --dtype f64 --iters 3; cd "$ROOT" ;;
    benchx:*)  # benchx:<tag>:<bench args with , for spaces> (no CPU leg)
      IFS=: read -r _ tag args <<< "$step"
      run "benchx_$tag" 600 python bench.py --no-cpu-baseline ${args//,/ } ;;
    tests:*)  # tests:<tag>:<limit s>:<pytest targets / args with , for spaces>
      IFS=: read -r _ tag lim targets <<< "$step"
      run "tests_$tag" "$lim" python -u -m pytest ${targets//,/ } -m gpu -v -x --timeout 300 --timeout-method thread -p no:cacheprovider -rf ;;
    testk:*)  # testk:<pytest -k expression with , for spaces>
      IFS=: read -r _ expr <<< "$step"
      run testk 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -p no:cacheprovider -rf -k "${expr//,/ }" ;;
    ab:*)  # ab:<tag>:<kprof_step args with , for spaces>:<variant names with ,> (tools/micro/ab.sh)
      IFS=: read -r _ tag args names <<< "$step"
      run "ab_$tag" 900 bash tools/micro/ab.sh "$OUT/ab_$tag.txt" "${args//,/ }" ${names//,/ } ;;
    probe:*)  # probe:<binary under tools/micro/v> (a stand-alone microbenchmark)
      IFS=: read -r _ name <<< "$step"
      run "probe_$name" 180 "tools/micro/v/$name" ;;
    py:*)  # py:<tag>:<script and args with , for spaces> (a python tool under its own limit)
      IFS=: read -r _ tag args <<< "$step"
      run "py_$tag" 300 python -u ${args//,/ } ;;
    profnet:*)  # profnet:<arch>[:compute] -> rocprofv3 kernel stats of the isolated network step
      IFS=: read -r _ arch comp <<< "$step"
      cd /tmp && run "profnet_${arch}" 300 rocprofv3 --kernel-trace --stats -d "$OUT/profnet_${arch}" -o run --output-format csv -- python "$ROOT/tools/kprof_net.py" --arch "$arch" --compute "${comp:-mfma}"; cd "$ROOT" ;;
    pmcnet:*)  # pmcnet:<arch>:<counters with ,> -> one PMC pass over the isolated network step
      IFS=: read -r _ arch ctrs <<< "$step"; tag="${arch}_$(echo "$ctrs" | tr ',' '_' | cut -c1-40)"
      cd /tmp && run "pmcnet_$tag" 180 rocprofv3 --kernel-trace --pmc ${ctrs//,/ } -d "$OUT/pmcnet_$tag" -o run --output-format csv -- python "$ROOT/tools/kprof_net.py" --arch "$arch" --compute mfma --iters 5; cd "$ROOT" ;;
    abnet:*)  # abnet:<tag>:<kprof_net args with , for spaces>:<variant names with ,> (isolated network step)
      IFS=: read -r _ tag args names <<< "$step"
      AB_SCRIPT=tools/kprof_net.py run "abnet_$tag" 900 bash tools/micro/ab.sh "$OUT/abnet_$tag.txt" "${args//,/ }" ${names//,/ } ;;
    pmcv:*)  # pmcv:<variant|default>:<kprof_step args with ,>:<counters with ,> -> one PMC pass
      IFS=: read -r _ var args ctrs <<< "$step"; tag="${var}_$(echo "$ctrs" | tr ',' '_' | cut -c1-40)_$(echo "$args" | md5sum | cut -c1-6)"
      if [ "$var" = default ]; then lib=$ROOT/spectralmc_amd/libspectralmc_hip.so; else lib=$ROOT/tools/micro/v/libsmc_$var.so; fi
      cd /tmp && SMC_LIB_PATH=$lib run "pmcv_$tag" 120 rocprofv3 --kernel-trace --pmc ${ctrs//,/ } -d "$OUT/pmcv_$tag" -o run --output-format csv -- python "$ROOT/tools/kprof_step.py" ${args//,/ }; cd "$ROOT" ;;
    testlib:*)  # testlib:<variant|default>:<pytest -k expression with , for spaces> (GPU tests on a variant library)
      IFS=: read -r _ var expr <<< "$step"
      if [ "$var" = default ]; then lib=$ROOT/spectralmc_amd/libspectralmc_hip.so; else lib=$ROOT/tools/micro/v/libsmc_$var.so; fi
      SMC_LIB_PATH=$lib run "testlib_$var" 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider -rf -k "${expr//,/ }" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "all steps done"
