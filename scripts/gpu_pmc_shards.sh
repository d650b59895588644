#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of rank 0's shard for C4 at W = 2, 4, 8 and C5 at W = 8
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1
for W in 2 4 8; do bash scripts/pmc_shard.sh $TAG C4 $W || exit $?; done
bash scripts/pmc_shard.sh $TAG C5 8 || exit $?
