#!/bin/bash
# Round 5: the reduce's range quantum (a tile, 512 containers, vs 256 / 64: more waves on
# small shards, every resident slot used); the harness checks identical totals.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05v}
mkdir -p gpurun_out
for SH in 8 4 2 1; do
  timeout -k 10 300 python3 -u scripts/ab_variants.py run --step --config C4 --shard $SH --rounds 7 --reps 20 base rq256 rq64 \
    > gpurun_out/ab_${TAG}_step_s$SH.txt 2>&1 || exit $?
  grep '^{' gpurun_out/ab_${TAG}_step_s$SH.txt
done
