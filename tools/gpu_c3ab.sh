#!/bin/bash
# GPU box: C3 parity tests, then the C3 timing (tools/bench_c3.py) of the default library vs
# variants/librabia_gpu_prev.so, interleaved 3 rounds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out; mkdir -p $OUT; cd $R
TAG=${1:-c3ab}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "cluster or c3" > $OUT/${TAG}_tests.log 2>&1 \
  || { echo "tests failed"; tail -30 $OUT/${TAG}_tests.log; exit 1; }
tail -1 $OUT/${TAG}_tests.log
for r in 1 2 3; do
  for v in default prev; do
    if [ $v = prev ]; then L=$R/rabia_amd/lib/variants/librabia_gpu_prev.so; else L=$R/rabia_amd/lib/librabia_gpu.so; fi
    RABIA_GPU_LIB=$L timeout -k 10 300 python tools/bench_c3.py --reps 5 > $OUT/${TAG}_${v}_$r.json 2> $OUT/${TAG}_${v}_$r.err \
      || { echo "bench_c3 failed"; tail -20 $OUT/${TAG}_${v}_$r.err; exit 1; }
    echo "$v $r $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print({k:v for k,v in d.items() if 'ms' in k or 'us' in k})" $OUT/${TAG}_${v}_$r.json)"
  done
done
