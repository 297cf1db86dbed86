#!/bin/bash
# VALU evidence for the C3 cluster kernel: one SQ/GRBM counter pass over
# tools/bench_c3.py (its own run, kernel trace only, under a hard time limit).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
  -d $OUT/pmc_c3 -o c3 --output-format csv -- python3 $R/tools/bench_c3.py --reps 3 > $OUT/pmc_c3.log 2>&1
rc=$?
tail -3 $OUT/pmc_c3.log
exit $rc
