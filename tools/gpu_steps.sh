#!/bin/bash
# GPU-box helper: run the named steps in order, each under its own time limit,
# stopping at the first failure. Steps:
#   kv      tests/test_kv.py (-m gpu)
#   c4      tests/test_full_size.py::test_c4_full_size_pipeline
#   gpu     the whole -m gpu suite
#   ab      tools/ab_variants.py with $AB_DIAGS (default: the round-1 tiled kernel vs the default)
#   c4b     tools/bench_c4.py
#   bench   python bench.py (default run)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu"
for s in "$@"; do
  case $s in
    kv)    timeout -k 10 600 $PT tests/test_kv.py > $OUT/pt_kv.log 2>&1 || { tail -40 $OUT/pt_kv.log; exit 1; }; tail -2 $OUT/pt_kv.log ;;
    c4)    timeout -k 10 600 $PT tests/test_full_size.py -k c4 > $OUT/pt_c4.log 2>&1 || { tail -40 $OUT/pt_c4.log; exit 1; }; tail -2 $OUT/pt_c4.log ;;
    gpu)   timeout -k 10 1100 $PT tests > $OUT/pt_gpu.log 2>&1 || { tail -40 $OUT/pt_gpu.log; exit 1; }; tail -2 $OUT/pt_gpu.log ;;
    ab)    AB_DIAGS=${AB_DIAGS:-legacy:0x10000} timeout -k 10 600 python tools/ab_variants.py > $OUT/ab_diag.json 2> $OUT/ab_diag.err || { tail -20 $OUT/ab_diag.err; exit 1; }; cat $OUT/ab_diag.json ;;
    c4b)   timeout -k 10 300 python tools/bench_c4.py --reps 5 > $OUT/c4.json 2>&1 || { tail -20 $OUT/c4.json; exit 1; }; cat $OUT/c4.json ;;
    bench) timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }; cat $OUT/bench.json ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
