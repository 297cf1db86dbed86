#!/bin/bash
# Experiment builds of librabia_gpu.so (A/B via RABIA_GPU_LIB, tools/ab_variants.py).
set -e
cd "$(dirname "$0")/.."
mkdir -p rabia_amd/lib/variants && rm -f rabia_amd/lib/variants/*.so
for v in "$@"; do
  name=${v%%:*}; defs=${v#*:}
  args=()
  for d in ${defs//;/ }; do args+=("-D$d"); done
  python -m rabia_amd.build --out=rabia_amd/lib/variants/librabia_gpu_$name.so "${args[@]}" > /dev/null
  echo built $name
done
