#!/bin/bash
# Round 5: the fit's priority by how far a workgroup is behind its segment's queue (pad)
# vs by progress quarters (base): step A/B, and the pad build's N = 1 / 8-way timelines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05s}
mkdir -p gpurun_out
for SH in 8 4 1; do
  timeout -k 10 300 python3 -u scripts/ab_variants.py run --step --config C4 --shard $SH --rounds 7 --reps 20 base pad \
    > gpurun_out/ab_${TAG}_step_s$SH.txt 2>&1 || exit $?
  grep '^{' gpurun_out/ab_${TAG}_step_s$SH.txt
done
for SH in 1 8; do
  timeout -k 10 200 python3 -u scripts/probe/timeline.py tla --config C4 --shard $SH --pipeline --dump gpurun_out/tl_${TAG}_s$SH.npy \
    > gpurun_out/tl_${TAG}_s$SH.txt 2>&1 || exit $?
  grep "fit loop" gpurun_out/tl_${TAG}_s$SH.txt
done
