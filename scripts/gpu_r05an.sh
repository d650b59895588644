#!/bin/bash
# Round 5: per-workgroup timeline of the 8-way C4 rank's step with node prep in the reduce
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05an}
mkdir -p gpurun_out
timeout -k 10 200 python3 -u scripts/probe/timeline.py tl --config C4 --shard 8 --pipeline --dump gpurun_out/tl_${TAG}_c4w8.npy \
  > gpurun_out/tl_${TAG}_c4w8.txt 2>&1 || exit $?
cat gpurun_out/tl_${TAG}_c4w8.txt | tail -40
