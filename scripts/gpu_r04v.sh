#!/bin/bash
# Round 4: per-workgroup timelines of the bench's pipeline (kcc_capacity_partial_async) at
# rank 0 of an 8-way C4 split (the clamp in the fit) and at C4 (-DKCC_TIMELINE variant).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04v}
mkdir -p gpurun_out
timeout -k 10 180 python -u scripts/probe/timeline.py tl --config C4 --shard 8 --pipeline > gpurun_out/tl_${TAG}_c4w8.txt 2>&1 || exit $?
cat gpurun_out/tl_${TAG}_c4w8.txt
timeout -k 10 180 python -u scripts/probe/timeline.py tl --config C4 --pipeline > gpurun_out/tl_${TAG}_c4.txt 2>&1 || exit $?
