#!/bin/bash
# Round 5: the fit's priority schemes — by progress quarters (base), boosted through the
# static first claim only (pm1), first claim then progress halves (pm2); step A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05q}
mkdir -p gpurun_out
for SH in 8 4 1; do
  timeout -k 10 300 python3 -u scripts/ab_variants.py run --step --config C4 --shard $SH --rounds 7 --reps 20 base pm1 pm2 \
    > gpurun_out/ab_${TAG}_step_s$SH.txt 2>&1 || exit $?
  grep '^{' gpurun_out/ab_${TAG}_step_s$SH.txt
done
