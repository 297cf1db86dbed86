#!/bin/bash
# One GPU-box session: parity tests, bench, rocprofv3 kernel trace, PMC traffic.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
TAG=${1:-r01}
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o bench --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 30 --warmup 5 > $OUT/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof_$TAG.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_$TAG -o pmc --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 10 --warmup 2 > $OUT/pmc_fetch_$TAG.log 2>&1 || { echo "pmc fetch failed"; tail -30 $OUT/pmc_fetch_$TAG.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write_$TAG -o pmc --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 10 --warmup 2 > $OUT/pmc_write_$TAG.log 2>&1 || { echo "pmc write failed"; tail -30 $OUT/pmc_write_$TAG.log; exit 1; }
cd $R
python3 tools/pmc_traffic.py $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG 5 1073741824 $OUT/pmc_c2.json || echo "pmc parse failed"
cat $OUT/prof_$TAG/bench_kernel_stats.csv | head -5
