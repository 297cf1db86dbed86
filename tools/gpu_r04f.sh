#!/bin/bash
# Round 4: the per-GPU cost of the N > 1 C2 path (one-shard pipeline vs the single
# evaluator) with a kernel trace; C5 lines at the 8-GPU shard size.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/r04f
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c2_single.json 2> $OUT/err.log &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --sharded > $OUT/c2_sharded.json 2>> $OUT/err.log &&
timeout -k 10 300 python bench.py --config c5 --c5-windows 8 --steps 20 --warmup 5 --sharded --no-cpu-baseline \
  > $OUT/c5_shard8x2e23.json 2>> $OUT/err.log &&
export TMPDIR=/tmp && cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c2s -o c2s --output-format csv -- \
  python3 $R/bench.py --steps 10 --warmup 3 --sharded --no-cpu-baseline > $OUT/prof_c2s.log 2>&1
