#!/bin/bash
# Round 4: per-phase stamps of the 512 x 4 lag kernel at 2^30 slots, and an interleaved
# A/B of default-policy plane stores against nt stores.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r04z
mkdir -p $OUT
cd $R
timeout -k 10 300 python tools/lag_stamps.py > $OUT/stamps.json 2> $OUT/stamps.err &&
AB_SLOTS=1073741824 AB_ROUNDS=4 timeout -k 10 600 python -u tools/ab_variants.py > $OUT/ab.json 2> $OUT/ab.err
