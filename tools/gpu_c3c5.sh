#!/bin/bash
# GPU box: C3 two-shard test, then the C3 and C5 bench lines (with CPU baselines) and
# the C5 step at the 8/4/2-GPU shard sizes (2^23..2^25 slots, n = 9) on one GPU.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
TAG=${1:-c35}
timeout -k 10 300 python -u -m pytest tests/test_full_size.py -m gpu -x -q --timeout 240 --timeout-method thread -k "c3" \
  > $OUT/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/${TAG}_tests.log; exit 1; }
tail -1 $OUT/${TAG}_tests.log
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 > $OUT/${TAG}_c3.json 2> $OUT/${TAG}_c3.err \
  || { echo "c3 bench failed"; tail -20 $OUT/${TAG}_c3.err; exit 1; }
cat $OUT/${TAG}_c3.json
timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 > $OUT/${TAG}_c5_64.json 2> $OUT/${TAG}_c5_64.err \
  || { echo "c5 bench failed"; tail -20 $OUT/${TAG}_c5_64.err; exit 1; }
cat $OUT/${TAG}_c5_64.json
for W in 8 16 32; do
  timeout -k 10 300 python bench.py --config c5 --c5-windows $W --steps 40 --warmup 5 --no-cpu-baseline \
    > $OUT/${TAG}_c5_$W.json 2> $OUT/${TAG}_c5_$W.err || { echo "c5 $W failed"; tail -20 $OUT/${TAG}_c5_$W.err; exit 1; }
  cat $OUT/${TAG}_c5_$W.json
done
