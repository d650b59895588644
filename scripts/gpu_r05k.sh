#!/bin/bash
# Round 5: the fit's issue priority by progress (fprio) vs base — step A/B at the C4 8-way /
# 4-way / 2-way ranks and C4, and the priority build's raw timeline at the 8-way rank.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05k}
mkdir -p gpurun_out
timeout -k 10 200 python3 -u scripts/probe/timeline.py tlp --config C4 --shard 8 --pipeline --dump gpurun_out/tl_${TAG}_p_c4w8.npy \
  > gpurun_out/tl_${TAG}_p_c4w8.txt 2>&1 || exit $?
grep "fit loop\|fit whole" gpurun_out/tl_${TAG}_p_c4w8.txt
for SH in 8 4 2 1; do
  timeout -k 10 300 python3 -u scripts/ab_variants.py run --step --config C4 --shard $SH --rounds 7 --reps 20 base fprio \
    > gpurun_out/ab_${TAG}_step_s$SH.txt 2>&1 || exit $?
  grep '^{' gpurun_out/ab_${TAG}_step_s$SH.txt
done
