#!/bin/bash
# Round 5: raw per-workgroup fit timeline at the C4 8-way rank (dumped for offline analysis).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05j}
mkdir -p gpurun_out
timeout -k 10 200 python3 -u scripts/probe/timeline.py tl --config C4 --shard 8 --pipeline --dump gpurun_out/tl_${TAG}_c4w8.npy \
  > gpurun_out/tl_${TAG}_c4w8.txt 2>&1 || exit $?
timeout -k 10 200 python3 -u scripts/probe/timeline.py tl --config C4 --shard 1 --pipeline --dump gpurun_out/tl_${TAG}_c4.npy \
  > gpurun_out/tl_${TAG}_c4.txt 2>&1 || exit $?
grep "fit" gpurun_out/tl_${TAG}_c4w8.txt | head -8
