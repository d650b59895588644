#!/bin/bash
# Round 5 diagnostics: the grids' resident counts, and per-workgroup timelines of the C4 step
# (one GPU) and of rank 0's 8-way shard (KCC_TIMELINE variant).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05c}
mkdir -p gpurun_out
timeout -k 10 120 python3 -u scripts/probe/occupancy.py > gpurun_out/occ_$TAG.txt 2>&1 || exit $?
cat gpurun_out/occ_$TAG.txt
timeout -k 10 200 python3 -u scripts/probe/timeline.py tl --config C4 --shard 1 --pipeline > gpurun_out/tl_${TAG}_c4.txt 2>&1 || exit $?
grep -v Warning gpurun_out/tl_${TAG}_c4.txt | tail -32
timeout -k 10 200 python3 -u scripts/probe/timeline.py tl --config C4 --shard 8 --pipeline > gpurun_out/tl_${TAG}_c4w8.txt 2>&1 || exit $?
grep -v Warning gpurun_out/tl_${TAG}_c4w8.txt | tail -32
