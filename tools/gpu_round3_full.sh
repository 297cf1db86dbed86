#!/bin/bash
# GPU box, round 3 record: -m gpu suite, smoke, bench (C2 headline), rocprofv3 kernel trace of the
# bench, FETCH/WRITE PMC passes of the C2 step (lag kernel) and of the C5 sharded step (8 x 2^23).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
TAG=${1:-r03}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/${TAG}_pytest.log 2>&1 \
  || { echo "pytest failed"; tail -30 $OUT/${TAG}_pytest.log; exit 1; }
tail -1 $OUT/${TAG}_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/${TAG}_smoke.log; exit 1; }
tail -1 $OUT/${TAG}_smoke.log
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o bench --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 30 --warmup 5 > $OUT/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -30 $OUT/prof_$TAG.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_$TAG -o pmc --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 6 --warmup 2 > $OUT/pmc_fetch_$TAG.log 2>&1 || { echo "pmc fetch failed"; tail -30 $OUT/pmc_fetch_$TAG.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write_$TAG -o pmc --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 6 --warmup 2 > $OUT/pmc_write_$TAG.log 2>&1 || { echo "pmc write failed"; tail -30 $OUT/pmc_write_$TAG.log; exit 1; }
C5="--config c5 --c5-sharded --c5-batch 8 --c5-windows 8 --no-cpu-baseline --steps 6 --warmup 2"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch_c5_$TAG -o pmc --output-format csv -- python3 $R/bench.py $C5 > $OUT/pmc_fetch_c5_$TAG.log 2>&1 || { echo "pmc c5 fetch failed"; tail -30 $OUT/pmc_fetch_c5_$TAG.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write_c5_$TAG -o pmc --output-format csv -- python3 $R/bench.py $C5 > $OUT/pmc_write_c5_$TAG.log 2>&1 || { echo "pmc c5 write failed"; tail -30 $OUT/pmc_write_c5_$TAG.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c5_$TAG -o c5 --output-format csv -- python3 $R/bench.py --config c5 --c5-sharded --c5-batch 8 --c5-windows 8 --no-cpu-baseline --steps 20 --warmup 3 > $OUT/prof_c5_$TAG.log 2>&1 || { echo "rocprof c5 failed"; tail -30 $OUT/prof_c5_$TAG.log; exit 1; }
cd $R
python3 tools/pmc_traffic.py $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG 5 1073741824 $OUT/pmc_c2_$TAG.json ref_lag_kernel || echo "pmc parse failed"
python3 tools/pmc_traffic.py $OUT/pmc_fetch_c5_$TAG $OUT/pmc_write_c5_$TAG 9 67108864 $OUT/pmc_c5_$TAG.json "ref_step_kernel<9" || echo "pmc c5 parse failed"
head -5 $OUT/prof_$TAG/bench_kernel_stats.csv
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err || { echo "bench failed"; tail -30 $OUT/${TAG}_bench.err; exit 1; }
cat $OUT/${TAG}_bench.json
