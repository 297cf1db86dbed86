#!/bin/bash
# GPU box: the whole -m gpu suite, then an interleaved A/B at 2^30 slots (default vs variants/ and AB_DIAGS).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
TAG=${1:-ck}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/${TAG}_pytest.log 2>&1 \
  || { echo "pytest failed"; tail -30 $OUT/${TAG}_pytest.log; exit 1; }
tail -1 $OUT/${TAG}_pytest.log
for S in ${AB_SIZES:-1073741824}; do
  AB_SLOTS=$S AB_DIAGS=${AB_DIAGS:-""} AB_ROUNDS=3 timeout -k 10 600 python -u tools/ab_variants.py \
    > $OUT/${TAG}_ab_$S.json 2> $OUT/${TAG}_ab_$S.err || { echo "A/B failed"; tail -30 $OUT/${TAG}_ab_$S.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k:(round(v['median_us'],1),v['same_as_default']) for k,v in d.items()})" $OUT/${TAG}_ab_$S.json $S
done
