#!/bin/bash
# GPU-box check of the persistent lag REF kernel: its parity tests, then an
# interleaved A/B against the tiled kernel (2^28 and 2^30 slots), then one bench line.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
TAG=${1:-lag}
timeout -k 10 900 python -u -m pytest tests/test_lag_kernel.py -m gpu -x -v --timeout 300 --timeout-method thread \
  > $OUT/${TAG}_tests.log 2>&1 || { echo "lag tests failed"; tail -60 $OUT/${TAG}_tests.log; exit 1; }
tail -3 $OUT/${TAG}_tests.log
for S in 268435456 1073741824; do
  AB_SLOTS=$S AB_DIAGS=${AB_DIAGS:-"tiled:0x100000,l1024:0x400000"} AB_ROUNDS=3 timeout -k 10 600 python -u tools/ab_variants.py \
    > $OUT/${TAG}_ab_$S.json 2> $OUT/${TAG}_ab_$S.err || { echo "A/B failed"; tail -30 $OUT/${TAG}_ab_$S.err; exit 1; }
  cat $OUT/${TAG}_ab_$S.json
done
if [ -z "$NOBENCH" ]; then
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err \
    || { echo "bench failed"; tail -30 $OUT/${TAG}_bench.err; exit 1; }
  cat $OUT/${TAG}_bench.json
fi
