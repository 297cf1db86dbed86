#!/bin/bash
# GPU box: lag-kernel phase stamps (2 x 512 and 1 x 1024 per CU) at 2^30 and 2^28 slots.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
TAG=${1:-st}
for d in 0 0x400000; do
  for S in 1073741824 268435456; do
    STAMP_SLOTS=$S timeout -k 10 300 python -u tools/lag_stamps.py $d > $OUT/${TAG}_${d}_${S}.json 2> $OUT/${TAG}_${d}_${S}.err \
      || { echo "stamps failed"; tail -20 $OUT/${TAG}_${d}_${S}.err; exit 1; }
    echo "== diag $d slots $S"; cat $OUT/${TAG}_${d}_${S}.json
  done
done
