#!/bin/bash
# VALU evidence for the C3 cluster kernel over tools/bench_c3.py: pass 1 the SQ/GRBM
# issue counters, pass 2 the VALU instruction mix (whichever of the candidate
# counters this rocprofv3 lists), each its own run with kernel trace only, under a
# hard time limit. usage: tools/pmc_c3.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04}
OUT=$R/gpurun_out/pmc_c3_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d $OUT/p1 -o c3 --output-format csv -- python3 $R/tools/bench_c3.py --reps 3 > $OUT/p1.log 2>&1 || exit 1
MIX=$(python3 - "$OUT/counters_list.txt" <<'PY'
import re, sys
text = open(sys.argv[1]).read()
cands = ["SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_CVT", "SQ_INSTS_VALU_TRANS_F32",
         "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM", "SQ_INSTS_BRANCH"]
have = [c for c in cands if re.search(r"\b" + c + r"\b", text)]
print(" ".join(have[:8]))
PY
)
echo "mix counters: $MIX"
if [ -n "$MIX" ]; then
  timeout -s KILL 180 rocprofv3 --pmc $MIX -d $OUT/p2 -o c3 --output-format csv -- python3 $R/tools/bench_c3.py --reps 3 \
    > $OUT/p2.log 2>&1 || exit 1
fi
exit 0
