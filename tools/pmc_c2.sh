#!/bin/bash
# SQ/GRBM counter pass over the C2 bench step (its own run, kernel trace only, hard time limit).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
TAG=${1:-pmc_c2sq}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE \
  -d $OUT/$TAG -o c2 --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/$TAG.log 2>&1
rc=$?
tail -2 $OUT/$TAG.log
exit $rc
