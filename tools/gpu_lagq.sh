#!/bin/bash
# GPU box: lag-kernel parity tests, phase stamps at 2^30, interleaved A/B vs the tiled
# kernel (2^30, 2^28), one bench line. Each step time-limited; stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
TAG=${1:-lq}
timeout -k 10 600 python -u -m pytest tests/test_lag_kernel.py tests/test_shard_ref.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > $OUT/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/${TAG}_tests.log; exit 1; }
tail -2 $OUT/${TAG}_tests.log
STAMP_SLOTS=1073741824 timeout -k 10 300 python -u tools/lag_stamps.py 0 > $OUT/${TAG}_stamps.json 2> $OUT/${TAG}_stamps.err \
  || { echo "stamps failed"; tail -20 $OUT/${TAG}_stamps.err; exit 1; }
cat $OUT/${TAG}_stamps.json
for S in ${AB_SIZES:-1073741824 268435456}; do
  AB_SLOTS=$S AB_DIAGS=${AB_DIAGS:-"tiled:0x100000"} AB_ROUNDS=3 timeout -k 10 600 python -u tools/ab_variants.py \
    > $OUT/${TAG}_ab_$S.json 2> $OUT/${TAG}_ab_$S.err || { echo "A/B failed"; tail -30 $OUT/${TAG}_ab_$S.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k:(round(v['median_us'],1),v['same_as_default']) for k,v in d.items()})" $OUT/${TAG}_ab_$S.json $S
done
if [ -z "$NOBENCH" ]; then
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/${TAG}_bench.json 2> $OUT/${TAG}_bench.err \
    || { echo "bench failed"; tail -30 $OUT/${TAG}_bench.err; exit 1; }
  cat $OUT/${TAG}_bench.json
fi
