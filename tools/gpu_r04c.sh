#!/bin/bash
# Round 4: kvstore suite + C4 timing/trace (sort v2); C3 parity (scheduler hash v2),
# C3 bench + counters; bench C2 N=1 (agreement on the timed lag-kernel output).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/r04c
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kv.py tests/test_full_size.py tests/test_gpu_parity.py \
  -k "kv or c4 or c3 or cluster" -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 &&
timeout -k 10 300 python tools/bench_c4.py > $OUT/c4.json 2> $OUT/c4.err &&
timeout -k 10 300 python tools/bench_c3.py > $OUT/c3.json 2> $OUT/c3.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err &&
bash tools/pmc_c3.sh r04c > $OUT/pmc_c3.log 2>&1 &&
export TMPDIR=/tmp && cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c4 -o c4 --output-format csv -- \
  python3 $R/tools/bench_c4.py --no-cpu --reps 10 > $OUT/prof_c4.log 2>&1
