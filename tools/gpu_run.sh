#!/bin/bash
# One parameterised GPU-box recipe: runs the named steps in order, each under its own
# time limit, and stops at the first failure (no step runs after a fault, abort or
# time limit). Results under gpurun_out/$TAG/.
#   usage: bash tools/gpu_run.sh TAG STEP [STEP ...]
#   steps:
#     tests[=EXPR]      python -m pytest tests -m gpu (-k EXPR)
#     smoke             __graft_entry__.smoke()
#     bench             bench.py (C2 headline, CPU leg included)
#     bench_sharded     bench.py --sharded (the N > 1 per-GPU pipeline on one GPU, RCCL world 1)
#     c3[=NAME] | c5 | c5_sharded   bench.py --config ... (NAME: an A/B label)
#     c4[=NAME]         tools/bench_c4.py (kvstore apply; NAME: an A/B label, no CPU leg)
#     probe_c5[=K]      tools/c5_probe.py, n = 9, K windows of 2^23 (default 32)
#     ab[=SLOTS]        tools/ab_variants.py (interleaved A/B, AB_DIAGS / RABIA_AB_LIBS from the env)
#     stamps            tools/lag_stamps.py (per-phase lag-kernel stamps at 2^30)
#     stamps_shard      the same for the sharded step
#     shard_probe       tools/shard_step_probe.py (plain vs sharded step alone, 2^30 slots)
#     latency           tools/latency_1m.py (single 2^20 window)
#     warm[=zero]       tools/warm_probe.py (launch-to-launch ramp; =zero: outputs zeroed first)
#     driver[=NAME]     bench.py exactly as the round-end driver runs it (--steps 20 --warmup 5)
#     gloo2             bench.py --gpus 2 --backend gloo (two ranks on the one GPU, a rehearsal)
#     prof[=ARGS]       rocprofv3 --kernel-trace --stats over bench.py ARGS (default: the C2 line)
#     pmc[=ARGS]        two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over bench.py ARGS
#     sq[=ARGS]         one SQ/GRBM counter pass over bench.py ARGS
#     pmc_c3            tools/pmc_c3.sh (the C3 cluster kernel's VALU counters, two passes)
#     prof_c4           rocprofv3 kernel trace over tools/bench_c4.py
#     bench_sharded_eager   bench_sharded with the exchange enqueued right behind its own step
#     line=ARGS         bench.py --steps 20 --warmup 10 ARGS (one bench line)
#     lib[=PATH]        later steps load another build (repo-relative; no PATH: the in-tree library)
#     gap[=LIB] | prof_gap    tools/gap_probe.py (gaps between step kernels by stream traffic; LIB: another
#                       build, repo-relative), plain / under rocprofv3
#   ARGS use ':' for spaces, e.g. prof=--config:c5:--sharded
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:?usage: gpu_run.sh TAG STEP...}
shift
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
export PYTHONUNBUFFERED=1
# the snapshot's prebuilt library as it is (through the /root/repo symlink, so the loader's
# staleness check against the sources, which may be newer mid-edit, does not rebuild it)
export RABIA_GPU_LIB=/root/repo/rabia_amd/lib/librabia_gpu.so

run() {  # name seconds command...
  local name=$1 secs=$2
  shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "$name failed (rc $rc)"
    tail -30 "$OUT/$name.err"
    tail -30 "$OUT/$name.out"
    exit $rc
  fi
  tail -2 "$OUT/$name.out"
}

prof_run() {  # name seconds rocprof-args... -- bench args (rocprofv3 needs the program itself after --)
  local name=$1 secs=$2
  shift 2
  echo "== $name"
  (export TMPDIR=/tmp; cd /tmp && timeout -s KILL "$secs" rocprofv3 "$@" > "$OUT/$name.log" 2>&1)
  local rc=$?
  if [ $rc -ne 0 ]; then
    echo "$name failed (rc $rc)"
    tail -30 "$OUT/$name.log"
    exit $rc
  fi
}

for step in "$@"; do
  name=${step%%=*}
  arg=""
  [ "$step" != "$name" ] && arg=${step#*=}
  bargs=${arg//:/ }
  sfx=$(echo "$arg" | tr -c 'a-zA-Z0-9\n' '_')  # per-argument output names
  case $name in
    tests)
      if [ -n "$arg" ]; then
        run tests 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${arg//:/ }"
      else
        run tests 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
      fi ;;
    smoke) run smoke 200 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 400 python bench.py ;;
    bench_sharded) run bench_sharded 300 python bench.py --sharded --steps 20 --warmup 10 --no-cpu-baseline ;;
    c3) run "c3$sfx" 300 python bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline ;;
    c5) run c5 300 python bench.py --config c5 --steps 20 --warmup 10 ;;
    c5_sharded) run c5_sharded 300 python bench.py --config c5 --sharded --steps 20 --warmup 10 ;;
    c4)
      if [ -n "$arg" ]; then run "c4_$sfx" 300 python tools/bench_c4.py --no-cpu
      else run c4 300 python tools/bench_c4.py; fi ;;
    probe_c5) run "probe_c5_${arg:-32}" 400 python tools/c5_probe.py --n 9 --window-log2 23 --k "${arg:-32}" --diags default:0 ;;
    ab) AB_SLOTS=${arg:-1073741824} AB_ROUNDS=${AB_ROUNDS:-4} run "ab_${arg:-1073741824}" 700 python -u tools/ab_variants.py ;;
    stamps) run stamps 300 python tools/lag_stamps.py ;;
    stamps_shard) STAMP_SHARD=1 run stamps_shard 300 python tools/lag_stamps.py ;;
    shard_probe) run shard_probe 300 python tools/shard_step_probe.py ;;
    latency) run "latency$sfx" 300 python tools/latency_1m.py ;;
    warm) run "warm$sfx" 300 env ${arg:+PROBE_ZERO=1} python tools/warm_probe.py ;;
    driver) run "driver$sfx" 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 ;;
    gloo2) run gloo2 300 python bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 --no-cpu-baseline ;;
    prof)
      prof_run "prof$sfx" 500 --kernel-trace --stats -d "$OUT/prof$sfx" -o run --output-format csv -- \
        python3 "$R/bench.py" --no-cpu-baseline --steps 30 --warmup 10 $bargs ;;
    pmc)
      prof_run "pmc_fetch$sfx" 240 --pmc FETCH_SIZE -d "$OUT/pmc_fetch$sfx" -o pmc --output-format csv -- \
        python3 "$R/bench.py" --no-cpu-baseline --steps 6 --warmup 2 $bargs
      prof_run "pmc_write$sfx" 240 --pmc WRITE_SIZE -d "$OUT/pmc_write$sfx" -o pmc --output-format csv -- \
        python3 "$R/bench.py" --no-cpu-baseline --steps 6 --warmup 2 $bargs ;;
    sq)
      prof_run "sq$sfx" 240 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
        SQ_INSTS_LDS GRBM_GUI_ACTIVE -d "$OUT/sq$sfx" -o sq --output-format csv -- \
        python3 "$R/bench.py" --no-cpu-baseline --steps 3 --warmup 1 $bargs ;;
    pmc_c3) run pmc_c3 500 bash tools/pmc_c3.sh "$TAG" ;;
    prof_c4)
      prof_run prof_c4 500 --kernel-trace --stats -d "$OUT/prof_c4" -o run --output-format csv -- \
        python3 "$R/tools/bench_c4.py" --no-cpu ;;
    bench_sharded_eager) run bench_sharded_eager 300 python bench.py --sharded --fixup-eager --steps 20 --warmup 10 \
      --no-cpu-baseline ;;
    lib) export RABIA_GPU_LIB="$R/${arg:-rabia_amd/lib/librabia_gpu.so}"; echo "== lib $RABIA_GPU_LIB" ;;
    line) run "line$sfx" 300 python bench.py --steps 20 --warmup 10 $bargs ;;
    gap)
      if [ -n "$arg" ]; then RABIA_GPU_LIB="$R/$arg" run "gap$sfx" 300 python tools/gap_probe.py
      else run gap 300 python tools/gap_probe.py; fi ;;
    prof_gap)
      if [ -n "$arg" ]; then export RABIA_GPU_LIB="$R/$arg"; fi
      prof_run "prof_gap$sfx" 300 --kernel-trace --stats -d "$OUT/prof_gap$sfx" -o run --output-format csv -- \
        python3 "$R/tools/gap_probe.py"
      export RABIA_GPU_LIB=/root/repo/rabia_amd/lib/librabia_gpu.so ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
done
echo "all steps ok"
