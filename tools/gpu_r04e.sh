#!/bin/bash
# Round 4: timelines of the C5-size launch (n = 9, 2^26 slots): tiled-kernel tile stamps,
# lag-kernel phase stamps (forced), a trivial-launch baseline; and the 2^20 window.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/r04e
mkdir -p $OUT
export PYTHONUNBUFFERED=1
STAMP_N=9 STAMP_SLOTS=67108864 timeout -k 10 200 python tools/stamps.py > $OUT/stamps_n9_2e26.json 2> $OUT/stamps.err &&
STAMP_N=9 STAMP_SLOTS=67108864 timeout -k 10 200 python tools/lag_stamps.py 0x200000 > $OUT/lag_stamps_n9_2e26.json 2>> $OUT/stamps.err &&
STAMP_N=5 STAMP_SLOTS=1048576 timeout -k 10 200 python tools/stamps.py > $OUT/stamps_n5_2e20.json 2>> $OUT/stamps.err &&
STAMP_N=5 STAMP_SLOTS=268435456 timeout -k 10 200 python tools/stamps.py > $OUT/stamps_n5_2e28.json 2>> $OUT/stamps.err
