#!/bin/bash
# Round 4: kvstore decode staged in LDS (all loads in flight): kv parity suite, then the
# C4 stage timing interleaved with the global-memory decode build, then a kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r04q
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd $R
V=$R/rabia_amd/lib/variants/librabia_gpu_decglobal.so
timeout -k 10 600 python -u -m pytest tests/test_kv.py tests/test_full_size.py -m gpu -x -v --timeout 300 --timeout-method thread -k "kv or C4 or c4" > $OUT/tests.log 2>&1 &&
for r in 1 2; do
  timeout -k 10 200 python tools/bench_c4.py --no-cpu >> $OUT/c4_staged.jsonl 2>> $OUT/c4.err &&
  RABIA_GPU_LIB=$V timeout -k 10 200 python tools/bench_c4.py --no-cpu >> $OUT/c4_global.jsonl 2>> $OUT/c4.err || exit 1
done &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o c4 --output-format csv -- python3 $R/tools/bench_c4.py --no-cpu --reps 10 > $OUT/prof.log 2>&1
