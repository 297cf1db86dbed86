#!/bin/bash
# bench lines: C2 (1 GPU, with CPU baselines), C5 (1 GPU), and a 2-rank gloo rehearsal
# of the sharded one-engine pipeline on the box's one GPU.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo "c2 failed"; tail -30 $OUT/bench_c2.err; exit 1; }
cat $OUT/bench_c2.json
timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { echo "c5 failed"; tail -30 $OUT/bench_c5.err; exit 1; }
cat $OUT/bench_c5.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --backend gloo --steps 6 --warmup 2 --windows 16 > $OUT/bench_gloo2.json 2> $OUT/bench_gloo2.err || { echo "gloo2 failed"; tail -30 $OUT/bench_gloo2.err; exit 1; }
cat $OUT/bench_gloo2.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29512 bench.py --backend gloo --config c5 --steps 6 --warmup 2 > $OUT/bench_gloo4_c5.json 2> $OUT/bench_gloo4_c5.err || { echo "gloo4 c5 failed"; tail -30 $OUT/bench_gloo4_c5.err; exit 1; }
cat $OUT/bench_gloo4_c5.json
