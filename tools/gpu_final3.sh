#!/bin/bash
# GPU box, end-of-round record: -m gpu suite, smoke, bench (C2) with CPU baseline, rocprof
# kernel trace of the bench, C3 and C5 lines, FETCH/WRITE PMC of the C2 step.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
TAG=${1:-r03f}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/${TAG}_pytest.log 2>&1 \
  || { echo "pytest failed"; tail -30 $OUT/${TAG}_pytest.log; exit 1; }
tail -1 $OUT/${TAG}_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/${TAG}_smoke.log; exit 1; }
tail -1 $OUT/${TAG}_smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err || { echo "bench failed"; tail -30 $OUT/${TAG}_bench.err; exit 1; }
cat $OUT/${TAG}_bench.json
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 > $OUT/${TAG}_c3.json 2> $OUT/${TAG}_c3.err || { echo "c3 failed"; tail -20 $OUT/${TAG}_c3.err; exit 1; }
timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 > $OUT/${TAG}_c5.json 2> $OUT/${TAG}_c5.err || { echo "c5 failed"; tail -20 $OUT/${TAG}_c5.err; exit 1; }
timeout -k 10 300 python bench.py --config c5 --c5-sharded --c5-batch 8 --c5-windows 8 --steps 20 --warmup 3 > $OUT/${TAG}_c5_shard8x2e23.json 2> $OUT/${TAG}_c5s.err || { echo "c5 sharded failed"; tail -20 $OUT/${TAG}_c5s.err; exit 1; }
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o bench --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 30 --warmup 5 > $OUT/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof_$TAG.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_$TAG -o pmc --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 6 --warmup 2 > $OUT/pmc_fetch_$TAG.log 2>&1 || { echo "pmc fetch failed"; tail -30 $OUT/pmc_fetch_$TAG.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write_$TAG -o pmc --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 6 --warmup 2 > $OUT/pmc_write_$TAG.log 2>&1 || { echo "pmc write failed"; tail -30 $OUT/pmc_write_$TAG.log; exit 1; }
cd $R
python3 tools/pmc_traffic.py $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG 5 1073741824 $OUT/pmc_c2_$TAG.json ref_lag_kernel || echo "pmc parse failed"
head -4 $OUT/prof_$TAG/bench_kernel_stats.csv
