#!/bin/bash
# Round 4: interleaved A/B of the 512 x 4 lag kernel with each lane's first 8 draws of a
# ChaCha pass read from LDS at once (the select loop then picks them from registers).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r04aa
mkdir -p $OUT
cd $R
AB_SLOTS=1073741824 AB_ROUNDS=4 timeout -k 10 600 python -u tools/ab_variants.py > $OUT/ab.json 2> $OUT/ab.err
