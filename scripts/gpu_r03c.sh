#!/bin/bash
# parity tests, then the C4 (8-way shard, whole) and C5 (8-way shard) kernel traces
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1
bash scripts/gpu_round.sh $TAG || exit $?
bash scripts/gpu_shard_trace.sh $TAG C5 8 || exit $?
