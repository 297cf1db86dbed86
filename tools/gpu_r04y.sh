#!/bin/bash
# Round 4 final check: the whole -m gpu suite, smoke(), the default bench line, the
# one-shard sharded line, and the fix-up probe under the default grid (2048) and 1024 / 4096.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r04y
mkdir -p $OUT
export PYTHONUNBUFFERED=1
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 &&
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err &&
timeout -k 10 300 python bench.py --sharded --steps 20 --warmup 10 --no-cpu-baseline > $OUT/c2_sharded.json 2>> $OUT/bench.err &&
for v in default fg1024 fg4096; do
  if [ $v = default ]; then L=$R/rabia_amd/lib/librabia_gpu.so; else L=$R/rabia_amd/lib/variants/librabia_gpu_$v.so; fi
  RABIA_GPU_LIB=$L timeout -k 10 300 python tools/fixup_probe.py > $OUT/fix_$v.json 2>> $OUT/fix.err || exit 1
done
