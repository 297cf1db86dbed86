#!/bin/bash
# A/B of the current build against rabia_amd/lib/ab/librabia_gpu_old.so (an earlier build of the
# library, selected through RABIA_GPU_LIB): GPU parity first, then interleaved bench runs.
set -o pipefail
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1 || { tail -30 gpurun_out/ab/pytest.log; exit 1; }
tail -1 gpurun_out/ab/pytest.log
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 50 --warmup 10 > gpurun_out/ab/new_$i.json || exit 1
  RABIA_GPU_LIB=$PWD/rabia_amd/lib/ab/librabia_gpu_old.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 50 --warmup 10 > gpurun_out/ab/old_$i.json || exit 1
done
python - <<'P'
import json
for v in ("new","old"):
    print(v, [round(json.load(open(f"gpurun_out/ab/{v}_{i}.json"))["roofline"]["kernel_avg_us"],1) for i in (1,2,3)])
P
timeout -k 10 120 python tools/latency_1m.py > gpurun_out/ab/lat_new.json || exit 1
RABIA_GPU_LIB=$PWD/rabia_amd/lib/ab/librabia_gpu_old.so timeout -k 10 120 python tools/latency_1m.py > gpurun_out/ab/lat_old.json || exit 1
python - <<'P'
import json
for v in ("new", "old"):
    d = json.load(open(f"gpurun_out/ab/lat_{v}.json"))["us_per_launch_median"]
    print("1M", v, {k: d[k] for k in ("auto", "auto_no_lookback", "auto_no_stats")})
P
