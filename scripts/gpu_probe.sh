#!/bin/bash
# Diagnostics on the GPU box (variants built on the CPU side first):
#   timeline of the C4 step and of its 8-way shard (variants/libkcc_tl.so), then the A/B
#   of the named variants at C4 and at the 8-way shard.
#   bash scripts/gpu_probe.sh <tag> <variant>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 180 python -u scripts/probe/timeline.py tl --config C4 > gpurun_out/tl_${TAG}_c4.txt 2>&1 || exit $?
timeout -k 10 180 python -u scripts/probe/timeline.py tl --config C4 --shard 8 > gpurun_out/tl_${TAG}_c4w8.txt 2>&1 || exit $?
if [ $# -gt 0 ]; then
  timeout -k 10 300 python -u scripts/ab_variants.py run --config C4 --rounds 5 --reps 10 "$@" \
    > gpurun_out/ab_${TAG}_c4.txt 2>&1 || exit $?
  timeout -k 10 300 python -u scripts/ab_variants.py run --config C4 --shard 8 --rounds 5 --reps 20 "$@" \
    > gpurun_out/ab_${TAG}_c4w8.txt 2>&1 || exit $?
fi
tail -n 30 gpurun_out/tl_${TAG}_c4.txt gpurun_out/tl_${TAG}_c4w8.txt
[ $# -gt 0 ] && cat gpurun_out/ab_${TAG}_c4.txt gpurun_out/ab_${TAG}_c4w8.txt
exit 0
