#!/bin/bash
# Round 4: bench lines after the per-rank device fix: default C2, the one-shard sharded
# line, the two-rank gloo rehearsal (spawned by bench.py) and C3.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r04ac
mkdir -p $OUT
export PYTHONUNBUFFERED=1
cd $R
timeout -k 10 400 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 python bench.py --sharded --steps 20 --warmup 10 --no-cpu-baseline > $OUT/c2_sharded.json 2>> $OUT/bench.err &&
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --steps 5 --warmup 3 --no-cpu-baseline > $OUT/c2_g2.json 2>> $OUT/bench.err &&
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c3.json 2>> $OUT/bench.err
