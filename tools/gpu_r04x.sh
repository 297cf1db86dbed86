#!/bin/bash
# Round 4: fix-up grid 2048 (default) vs 1024 / 4096 workgroups, unrolled partials fold:
# shard parity tests, then the fix-up probe per build (interleaved twice) and a kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r04x
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_shard_ref.py tests/test_kv.py -k "shard or Shard or sharded or two_process or pipelined or records or follower" \
  -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 &&
for r in 1 2; do
  for v in default fg1024 fg4096; do
    if [ $v = default ]; then L=$R/rabia_amd/lib/librabia_gpu.so; else L=$R/rabia_amd/lib/variants/librabia_gpu_$v.so; fi
    RABIA_GPU_LIB=$L timeout -k 10 300 python tools/fixup_probe.py > $OUT/fix_${v}_$r.json 2>> $OUT/fix.err || exit 1
  done
done &&
cd /tmp && timeout -s KILL 240 rocprofv3 --kernel-trace --stats -d $OUT/fix_trace -o fix --output-format csv -- \
  python3 $R/tools/fixup_probe.py > $OUT/fixup_trace.json 2>> $OUT/fix.err
