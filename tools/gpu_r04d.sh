#!/bin/bash
# Round 4: kv sort v3 + C3 (LDS-staged states) parity, C4/C3 timing, C3 counters,
# C5 launch shapes in isolation.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/r04d
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kv.py tests/test_full_size.py tests/test_gpu_parity.py \
  -k "kv or c4 or c3 or cluster" -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 &&
timeout -k 10 300 python tools/bench_c4.py --no-cpu > $OUT/c4.json 2> $OUT/c4.err &&
timeout -k 10 300 python tools/bench_c3.py > $OUT/c3.json 2> $OUT/c3.err &&
timeout -k 10 300 python tools/c5_probe.py > $OUT/c5_probe.json 2> $OUT/c5_probe.err &&
timeout -k 10 300 python tools/c5_probe.py --n 5 --window-log2 24 --k 8 > $OUT/c5_probe_n5.json 2> $OUT/c5_probe_n5.err &&
bash tools/pmc_c3.sh r04d > $OUT/pmc_c3.log 2>&1 &&
export TMPDIR=/tmp && cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c4 -o c4 --output-format csv -- \
  python3 $R/tools/bench_c4.py --no-cpu --reps 10 > $OUT/prof_c4.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c5 -o c5 --output-format csv -- \
  python3 $R/tools/c5_probe.py --reps 10 > $OUT/prof_c5.log 2>&1
