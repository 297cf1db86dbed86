#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
OUT=$R/gpurun_out/r04g
mkdir -p $OUT
timeout -k 10 300 python tools/fixup_probe.py > $OUT/fixup.json 2> $OUT/fixup.err &&
export TMPDIR=/tmp && cd /tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o fx --output-format csv -- \
  python3 $R/tools/fixup_probe.py > $OUT/prof.log 2>&1
