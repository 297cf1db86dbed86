#!/bin/bash
# Round 4: draw records built in the draw loop (parity + step cost vs no records), and the
# fix-up's kernels under a kernel trace (which of its launches holds the time).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r04j
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_shard_ref.py tests/test_lag_shapes.py -k "shard or Shard or sharded or two_process or pipelined or records" \
  -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 &&
timeout -k 10 300 python tools/shard_step_probe.py > $OUT/shard_probe.json 2> $OUT/probe.err &&
RABIA_GPU_LIB=$R/rabia_amd/lib/variants/librabia_gpu_norec.so timeout -k 10 300 python tools/shard_step_probe.py \
  > $OUT/shard_probe_norec.json 2>> $OUT/probe.err &&
cd /tmp &&
timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/fix_trace -o fix --output-format csv -- \
  python3 $R/tools/fixup_probe.py > $OUT/fixup.json 2> $OUT/fixup.err &&
cd $R && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --sharded --no-cpu-baseline > $OUT/c2_sharded.json 2> $OUT/err.log
