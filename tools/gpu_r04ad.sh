#!/bin/bash
# Round 4 closing check (engine default device): the whole -m gpu suite, smoke(), the default
# bench line and the one-shard sharded line on the committed library.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r04ad
mkdir -p $OUT
export PYTHONUNBUFFERED=1
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 python bench.py --sharded --steps 20 --warmup 10 --no-cpu-baseline > $OUT/c2_sharded.json 2>> $OUT/bench.err
