#!/bin/bash
# Round 4 records for the 512 x 4 lag shape: C2 single and one-shard sharded kernel traces
# and HBM traffic passes (the C5 records are unchanged: its launches run the tiled kernel).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r04u
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $R/bench.py"
run() {  # tag, extra rocprof args, bench args
  local tag=$1; shift; local pr=$1; shift
  timeout -s KILL 240 rocprofv3 $pr -d $OUT/$tag -o $tag --output-format csv -- $B "$@" > $OUT/$tag.log 2>&1
}
run c2_trace "--kernel-trace --stats" --steps 20 --warmup 25 --no-cpu-baseline &&
run c2_fetch "--pmc FETCH_SIZE" --steps 5 --warmup 2 --no-cpu-baseline &&
run c2_write "--pmc WRITE_SIZE" --steps 5 --warmup 2 --no-cpu-baseline &&
run c2s_trace "--kernel-trace --stats" --sharded --steps 20 --warmup 10 --no-cpu-baseline &&
run c2s_fetch "--pmc FETCH_SIZE" --sharded --steps 5 --warmup 2 --no-cpu-baseline &&
run c2s_write "--pmc WRITE_SIZE" --sharded --steps 5 --warmup 2 --no-cpu-baseline &&
cd $R && python tools/pmc_traffic.py $OUT/c2_fetch $OUT/c2_write 5 1073741824 $OUT/pmc_c2.json &&
python tools/pmc_traffic.py $OUT/c2s_fetch $OUT/c2s_write 5 1073741824 $OUT/pmc_c2_sharded.json
