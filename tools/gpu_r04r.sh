#!/bin/bash
# Round 4: bench.py --gpus 2 rehearsal on one GPU (gloo, the ranks spawned by bench.py),
# and the C5 lines (single 2^26 step; the 8-GPU per-rank shard shape at N = 1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r04r
mkdir -p $OUT
export PYTHONUNBUFFERED=1
cd $R
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --steps 5 --warmup 3 --no-cpu-baseline > $OUT/c2_g2.json 2> $OUT/g2.err &&
timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 10 --no-cpu-baseline > $OUT/c5.json 2> $OUT/c5.err &&
timeout -k 10 300 python bench.py --config c5 --c5-windows 8 --sharded --steps 20 --warmup 10 --no-cpu-baseline > $OUT/c5s.json 2>> $OUT/c5.err
