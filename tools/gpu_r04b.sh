#!/bin/bash
# Round 4: lag-shape overflow test, C4 timing + kernel trace (hand-written sort),
# bench N=1, bench --gpus 2 gloo rehearsal.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/r04b
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_lag_shapes.py -x -v --timeout 200 --timeout-method thread \
  -k "overflow" > $OUT/lag_overflow.log 2>&1 &&
timeout -k 10 300 python tools/bench_c4.py > $OUT/c4.json 2> $OUT/c4.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 --no-cpu-baseline \
  > $OUT/bench_g2.json 2> $OUT/bench_g2.err &&
export TMPDIR=/tmp && cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c4 -o c4 --output-format csv -- \
  python3 $R/tools/bench_c4.py --no-cpu --reps 10 > $OUT/prof_c4.log 2>&1
