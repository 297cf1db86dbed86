#!/bin/bash
# GPU-box C4 session: the kvstore parity tests, then the C4 pipeline timing (default
# sort width and a bucket-width sweep) and a rocprofv3 kernel trace of the default.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-c4}
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_kv.py tests/test_full_size.py -m gpu -x -v --timeout 300 --timeout-method thread -k "kv or C4 or c4" > $OUT/pytest_kv.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_kv.log; exit 1; }
tail -3 $OUT/pytest_kv.log
timeout -k 10 300 python tools/bench_c4.py > $OUT/${TAG}.json 2> $OUT/${TAG}.err || { echo "bench_c4 failed"; tail -30 $OUT/${TAG}.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/${TAG}.json')); print(d['stage_us_median'], d['apply_warm_us_median'], d['cpu_baseline']['sample'][-40:])"
for bb in ${BUCKETS:-}; do
  timeout -k 10 200 python tools/bench_c4.py --no-cpu --bucket-bits $bb >> $OUT/${TAG}_sweep.jsonl 2>> $OUT/${TAG}.err || { echo "sweep $bb failed"; exit 1; }
done
[ -n "${BUCKETS:-}" ] && cat $OUT/${TAG}_sweep.jsonl
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o c4 --output-format csv -- python3 $R/tools/bench_c4.py --no-cpu --reps 10 > $OUT/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof_$TAG.log; exit 1; }
cut -d, -f1-4 $OUT/prof_$TAG/c4_kernel_stats.csv | cut -c1-160 | head -14
