#!/bin/bash
# GPU box: shard tests (multi-window launch == per-window), then the C5 sharded pipeline on
# one GPU at the 8/4/2/1-GPU shard sizes (2^23..2^26 slots per window, n = 9), with 1 and 8
# windows per shard launch.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
TAG=${1:-c5b}
timeout -k 10 600 python -u -m pytest tests/test_shard_ref.py tests/test_lag_kernel.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/${TAG}_tests.log; exit 1; }
tail -1 $OUT/${TAG}_tests.log
for B in ${BATCHES:-1 8}; do
  for W in ${WINS:-8 16 32 64}; do
    timeout -k 10 300 python bench.py --config c5 --c5-sharded --c5-batch $B --c5-windows $W --steps 20 --warmup 3 --no-cpu-baseline \
      > $OUT/${TAG}_b${B}_w$W.json 2> $OUT/${TAG}_b${B}_w$W.err || { echo "c5 b$B w$W failed"; tail -20 $OUT/${TAG}_b${B}_w$W.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('batch', sys.argv[2], 'win', sys.argv[3], 'launch_us', round(r['kernel_avg_us'],1), 'frac', round(r['frac'],3), 'ms_per_step', round(d['ms_per_step'],4), 'value', '%.3g' % d['value'])" $OUT/${TAG}_b${B}_w$W.json $B $W
  done
done
