#!/bin/bash
# Round 4: the fix-up as one thread per ChaCha12 block (atomic XOR patches, no segment
# pass): parity, kernel trace, A/B against the per-segment build, the one-shard C2 pipeline.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r04m
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_shard_ref.py tests/test_lag_shapes.py -k "shard or Shard or sharded or two_process or pipelined or records" \
  -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 &&
RABIA_GPU_LIB=$R/rabia_amd/lib/variants/librabia_gpu_fixseg.so timeout -k 10 300 python tools/fixup_probe.py > $OUT/fixup_seg.json 2> $OUT/fixup.err &&
timeout -k 10 300 python tools/fixup_probe.py > $OUT/fixup_blk.json 2>> $OUT/fixup.err &&
cd /tmp &&
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/fix_trace -o fix --output-format csv -- \
  python3 $R/tools/fixup_probe.py > $OUT/fixup_trace.json 2>> $OUT/fixup.err &&
cd $R && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --sharded --no-cpu-baseline > $OUT/c2_sharded.json 2> $OUT/err.log &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --sharded --no-cpu-baseline --fixup-stream fix > $OUT/c2_sharded_fix.json 2>> $OUT/err.log
