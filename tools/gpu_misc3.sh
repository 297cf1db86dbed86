#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
TAG=${1:-m3}
timeout -k 10 600 python -u -m pytest tests/test_shard_ref.py tests/test_kv.py tests/test_lag_kernel.py -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/${TAG}_tests.log 2>&1 \
  || { echo "tests failed"; tail -30 $OUT/${TAG}_tests.log; exit 1; }
tail -1 $OUT/${TAG}_tests.log
AB_SLOTS=1073741824 AB_ROUNDS=3 timeout -k 10 600 python -u tools/ab_variants.py > $OUT/${TAG}_ab.json 2> $OUT/${TAG}_ab.err || { echo "A/B failed"; tail -20 $OUT/${TAG}_ab.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print({k:(round(v['median_us'],1),v['same_as_default']) for k,v in d.items()})" $OUT/${TAG}_ab.json
