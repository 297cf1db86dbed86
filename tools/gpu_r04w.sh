#!/bin/bash
# Round 4: the sharded step (draw records) as 512 x 4 (default) vs 1024 x 2, alone on the
# GPU at the bench shape (tools/shard_step_probe.py, two passes each, interleaved).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r04w
mkdir -p $OUT
cd $R
V=$R/rabia_amd/lib/variants/librabia_gpu_shw2.so
for r in 1 2; do
  timeout -k 10 300 python tools/shard_step_probe.py >> $OUT/probe_w4.jsonl 2>> $OUT/probe.err &&
  RABIA_GPU_LIB=$V timeout -k 10 300 python tools/shard_step_probe.py >> $OUT/probe_w2.jsonl 2>> $OUT/probe.err || exit 1
done
