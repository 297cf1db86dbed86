#!/bin/bash
# Round 4: kvstore decode staged in LDS: the kv parity suite and C4 pipeline, the C4
# stage timing and its kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r04p
mkdir -p $OUT
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cd $R
timeout -k 10 600 python -u -m pytest tests/test_kv.py tests/test_full_size.py -m gpu -x -v --timeout 300 --timeout-method thread -k "kv or C4 or c4" > $OUT/tests.log 2>&1 &&
timeout -k 10 300 python tools/bench_c4.py > $OUT/c4.json 2> $OUT/c4.err &&
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o c4 --output-format csv -- python3 $R/tools/bench_c4.py --no-cpu --reps 10 > $OUT/prof.log 2>&1
