#!/bin/bash
# Round 4, first GPU pass: the lag-kernel shape tests, the kvstore suite (hand-written
# sort), a short bench (1 GPU) and the two-rank gloo rehearsal of bench.py --gpus 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/r04a
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kv.py tests/test_full_size.py -k "kv or c4" -x -v --timeout 200 \
  --timeout-method thread > $OUT/kv.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests/test_lag_shapes.py -x -v --timeout 400 --timeout-method thread \
  > $OUT/lag_shapes.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 --no-cpu-baseline \
  > $OUT/bench_g2.json 2> $OUT/bench_g2.err
