#!/bin/bash
# A/B of variants/ builds at C4 and its 8-way shard (one process each, interleaved rounds)
#   bash scripts/gpu_ab.sh <tag> <variant>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ab_variants.py run --config C4 --rounds 5 --reps 10 "$@" > gpurun_out/ab_${TAG}_c4.txt 2>&1 || exit $?
timeout -k 10 300 python -u scripts/ab_variants.py run --config C4 --shard 8 --rounds 5 --reps 20 "$@" > gpurun_out/ab_${TAG}_c4w8.txt 2>&1 || exit $?
grep -h '^{' gpurun_out/ab_${TAG}_c4.txt gpurun_out/ab_${TAG}_c4w8.txt
