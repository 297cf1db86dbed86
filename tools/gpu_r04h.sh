#!/bin/bash
# Round 4: segment fix-up (parity, isolation), the one-shard C2 pipeline (fix-up on the
# compute stream / on the second stream) vs the single evaluator, and the sharded step
# with / without its record stores (experiment build).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/r04h
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_shard_ref.py tests/test_lag_shapes.py -k "shard or Shard or sharded or two_process or pipelined or records" \
  -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 &&
timeout -k 10 300 python tools/fixup_probe.py > $OUT/fixup.json 2> $OUT/fixup.err &&
timeout -k 10 300 python tools/shard_step_probe.py > $OUT/shard_probe.json 2> $OUT/probe.err &&
RABIA_GPU_LIB=$R/rabia_amd/lib/variants/librabia_gpu_norec.so timeout -k 10 300 python tools/shard_step_probe.py \
  > $OUT/shard_probe_norec.json 2>> $OUT/probe.err &&
RABIA_GPU_LIB=$R/rabia_amd/lib/variants/librabia_gpu_direct.so timeout -k 10 300 python tools/shard_step_probe.py \
  > $OUT/shard_probe_direct.json 2>> $OUT/probe.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --sharded --no-cpu-baseline > $OUT/c2_sharded_comp.json 2> $OUT/err.log &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --sharded --no-cpu-baseline --fixup-stream fix > $OUT/c2_sharded_fix.json 2>> $OUT/err.log &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c2_single.json 2>> $OUT/err.log
