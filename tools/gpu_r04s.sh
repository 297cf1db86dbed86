#!/bin/bash
# Round 4: interleaved A/B of the lag kernel as 512 threads x 4 words (b128 plane loads) and
# with default-policy plane loads
# against the default 1024 x 2, at the bench shape.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r04s
mkdir -p $OUT
cd $R
AB_SLOTS=1073741824 AB_ROUNDS=4 timeout -k 10 600 python -u tools/ab_variants.py > $OUT/ab.json 2> $OUT/ab.err
