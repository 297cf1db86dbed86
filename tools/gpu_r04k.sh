#!/bin/bash
# Round 4: fix-up and follower statistics as per-workgroup partials (no same-address
# atomics): parity, the fix-up kernel trace, the one-shard C2 pipeline on both fix-up streams.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r04k
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_shard_ref.py tests/test_lag_shapes.py tests/test_kv.py tests/test_checkpoint.py tests/test_gpu_parity.py -k "shard or Shard or sharded or two_process or pipelined or records or follower or checkpoint" \
  -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 &&
cd /tmp &&
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/fix_trace -o fix --output-format csv -- \
  python3 $R/tools/fixup_probe.py > $OUT/fixup.json 2> $OUT/fixup.err &&
cd $R && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --sharded --no-cpu-baseline > $OUT/c2_sharded.json 2> $OUT/err.log &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --sharded --no-cpu-baseline --fixup-stream fix > $OUT/c2_sharded_fix.json 2>> $OUT/err.log
