#!/bin/bash
# Round 4 records: C2 headline kernel trace + HBM traffic passes (single and one-shard
# sharded step); C5 (single 2^26 step and
# the 8 x 2^23 shard pipeline) kernel traces + traffic passes. Each rocprofv3 pass its own
# run under a hard limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r04i
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $R/bench.py"
run() {  # tag, extra rocprof args, bench args
  local tag=$1; shift; local pr=$1; shift
  timeout -s KILL 240 rocprofv3 $pr -d $OUT/$tag -o $tag --output-format csv -- $B "$@" > $OUT/$tag.log 2>&1
}
run c2_trace "--kernel-trace --stats" --steps 20 --warmup 5 --no-cpu-baseline &&
run c2_fetch "--pmc FETCH_SIZE" --steps 5 --warmup 2 --no-cpu-baseline &&
run c2_write "--pmc WRITE_SIZE" --steps 5 --warmup 2 --no-cpu-baseline &&
run c2s_trace "--kernel-trace --stats" --sharded --steps 20 --warmup 5 --no-cpu-baseline &&
run c2s_fetch "--pmc FETCH_SIZE" --sharded --steps 5 --warmup 2 --no-cpu-baseline &&
run c2s_write "--pmc WRITE_SIZE" --sharded --steps 5 --warmup 2 --no-cpu-baseline &&
run c5_trace "--kernel-trace --stats" --config c5 --steps 20 --warmup 5 --no-cpu-baseline &&
run c5_fetch "--pmc FETCH_SIZE" --config c5 --steps 5 --warmup 2 --no-cpu-baseline &&
run c5_write "--pmc WRITE_SIZE" --config c5 --steps 5 --warmup 2 --no-cpu-baseline &&
run c5s_trace "--kernel-trace --stats" --config c5 --c5-windows 8 --sharded --steps 20 --warmup 5 --no-cpu-baseline &&
run c5s_fetch "--pmc FETCH_SIZE" --config c5 --c5-windows 8 --sharded --steps 5 --warmup 2 --no-cpu-baseline &&
run c5s_write "--pmc WRITE_SIZE" --config c5 --c5-windows 8 --sharded --steps 5 --warmup 2 --no-cpu-baseline &&
cd $R && python tools/pmc_traffic.py $OUT/c2_fetch $OUT/c2_write 5 1073741824 $OUT/pmc_c2.json &&
python tools/pmc_traffic.py $OUT/c2s_fetch $OUT/c2s_write 5 1073741824 $OUT/pmc_c2_sharded.json &&
python tools/pmc_traffic.py $OUT/c5_fetch $OUT/c5_write 9 67108864 $OUT/pmc_c5.json &&
python tools/pmc_traffic.py $OUT/c5s_fetch $OUT/c5s_write 9 67108864 $OUT/pmc_c5_sharded.json
