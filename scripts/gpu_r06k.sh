#!/bin/bash
# Round 6: the reduce's next-tile loads issued before the pending-block stores (lf: no
# vmcnt wait at the loop head before the prefetch) against the release order, C4 and its
# 8-way shard, then the whole step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06k}
bash scripts/gpu_ab.sh $TAG rel lf || exit $?
timeout -k 10 300 python -u scripts/ab_variants.py run --step --config C4 --rounds 7 --reps 10 rel lf > gpurun_out/ab_${TAG}_step.txt 2>&1 || exit $?
grep -h '^{' gpurun_out/ab_${TAG}_step.txt
