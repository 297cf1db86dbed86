#!/bin/bash
# Round 4: interleaved A/B of the 512 x 4 lag kernel with the next tile's round-2 loads issued
# before the decisions (two register sets) against the default, at the bench shape.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r04v
mkdir -p $OUT
cd $R
AB_SLOTS=1073741824 AB_ROUNDS=4 timeout -k 10 600 python -u tools/ab_variants.py > $OUT/ab.json 2> $OUT/ab.err
