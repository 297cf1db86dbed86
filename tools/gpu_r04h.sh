#!/bin/bash
# Round 4: segment fix-up: shard parity suites, the fix-up in isolation, the one-shard C2
# pipeline (fix-up on the compute stream / on the second stream) vs the single evaluator.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/r04h
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_shard_ref.py tests/test_lag_shapes.py -k "shard or Shard or sharded or two_process or pipelined or records" \
  -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 &&
timeout -k 10 300 python tools/fixup_probe.py > $OUT/fixup.json 2> $OUT/fixup.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --sharded --no-cpu-baseline > $OUT/c2_sharded_comp.json 2> $OUT/err.log &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --sharded --no-cpu-baseline --fixup-stream fix > $OUT/c2_sharded_fix.json 2>> $OUT/err.log &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c2_single.json 2>> $OUT/err.log &&
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --steps 4 --warmup 2 --no-cpu-baseline > $OUT/c2_g2.json 2>> $OUT/err.log
