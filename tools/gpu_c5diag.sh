#!/bin/bash
# GPU box: the C5 shard step at 2^23..2^26 slots (n = 9, one GPU) under rg_debug_set switches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
TAG=${1:-c5d}
for D in ${DIAGS:-0 0x100000 0x400000}; do
  for W in ${WINS:-8 16 64}; do
    timeout -k 10 300 python bench.py --config c5 --c5-windows $W --steps 40 --warmup 5 --no-cpu-baseline --diag $D \
      > $OUT/${TAG}_${D}_$W.json 2> $OUT/${TAG}_${D}_$W.err || { echo "c5 $D $W failed"; tail -20 $OUT/${TAG}_${D}_$W.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], round(d['roofline']['kernel_avg_us'],1), round(d['ms_per_step']*1000,1))" $OUT/${TAG}_${D}_$W.json $D $W
  done
done
