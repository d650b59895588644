#!/bin/bash
# Round 5: the clamp-value prefetch A/B, then the 8-way rank's timeline with node prep's
# row phases stamped
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05ap}
mkdir -p gpurun_out
SKIP_TESTS=1 bash scripts/gpu_r05ad.sh $TAG || exit $?
timeout -k 10 200 python3 -u scripts/probe/timeline.py tl --config C4 --shard 8 --pipeline --dump gpurun_out/tl_${TAG}_c4w8.npy \
  > gpurun_out/tl_${TAG}_c4w8.txt 2>&1 || exit $?
head -20 gpurun_out/tl_${TAG}_c4w8.txt
