#!/bin/bash
# GPU box, round 3: the -m gpu suite, an interleaved A/B of the REF step shapes at
# 2^30 slots, then one bench line (with the CPU baseline). Every GPU step has its own
# time limit; the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
TAG=${1:-r3}
K=${2:-}
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${KARG[@]}" \
  > $OUT/${TAG}_tests.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/${TAG}_tests.log; exit 1; }
tail -3 $OUT/${TAG}_tests.log
if [ -z "$NOAB" ]; then
  for S in ${AB_SIZES:-1073741824}; do
    AB_SLOTS=$S AB_DIAGS=${AB_DIAGS:-"l512:0x400000,tiled:0x100000"} AB_ROUNDS=3 timeout -k 10 600 \
      python -u tools/ab_variants.py > $OUT/${TAG}_ab_$S.json 2> $OUT/${TAG}_ab_$S.err \
      || { echo "A/B failed"; tail -30 $OUT/${TAG}_ab_$S.err; exit 1; }
    cat $OUT/${TAG}_ab_$S.json
  done
fi
if [ -z "$NOBENCH" ]; then
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err \
    || { echo "bench failed"; tail -30 $OUT/${TAG}_bench.err; exit 1; }
  cat $OUT/${TAG}_bench.json
fi
