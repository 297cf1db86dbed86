#!/bin/bash
# HBM traffic of the C4 kvstore kernels: FETCH_SIZE and WRITE_SIZE passes (separate
# runs, kernel trace only, hard time limits) over tools/bench_c4.py --reps 1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_c4_fetch -o c4 --output-format csv -- python3 $R/tools/bench_c4.py --reps 1 > $OUT/pmc_c4_fetch.log 2>&1 || { tail -5 $OUT/pmc_c4_fetch.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_c4_write -o c4 --output-format csv -- python3 $R/tools/bench_c4.py --reps 1 > $OUT/pmc_c4_write.log 2>&1 || { tail -5 $OUT/pmc_c4_write.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $OUT/pmc_c4_sq -o c4 --output-format csv -- python3 $R/tools/bench_c4.py --reps 1 > $OUT/pmc_c4_sq.log 2>&1 || { tail -5 $OUT/pmc_c4_sq.log; exit 1; }
echo done
