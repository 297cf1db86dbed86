#!/bin/bash
# GPU-box A/B of kvstore sort variants (tools/build_variants.sh builds): the kv GPU
# tests under each variant, then interleaved bench_c4 runs. Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
for v in "$@"; do
  RABIA_GPU_LIB=$R/rabia_amd/lib/variants/librabia_gpu_$v.so timeout -k 10 300 python -u -m pytest tests/test_kv.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/ab_sort_test_$v.log 2>&1 || { echo "tests failed for $v"; tail -30 $OUT/ab_sort_test_$v.log; exit 1; }
  echo "$v: $(tail -1 $OUT/ab_sort_test_$v.log)"
done
for round in 1 2; do
  timeout -k 10 200 python tools/bench_c4.py --no-cpu --reps 5 | sed "s/^/{\"lib\": \"default\", \"r\": $round, \"d\": /; s/$/}/" >> $OUT/ab_sort.jsonl || exit 1
  for v in "$@"; do
    RABIA_GPU_LIB=$R/rabia_amd/lib/variants/librabia_gpu_$v.so timeout -k 10 200 python tools/bench_c4.py --no-cpu --reps 5 | sed "s/^/{\"lib\": \"$v\", \"r\": $round, \"d\": /; s/$/}/" >> $OUT/ab_sort.jsonl || exit 1
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/ab_sort.jsonl"):
    d = json.loads(l)
    print(d["lib"], d["r"], round(d["d"]["stage_us_median"]["apply"], 1), round(d["d"]["apply_warm_us_median"], 1), d["d"]["store"]["ordered_batches"], d["d"]["store"]["flags"])
PY
