#!/bin/bash
# Round 6: the reduce's waves in 2 / 3 rounds of the resident slots (range halved / a third:
# the dispatcher refills a finished workgroup's slot) against one round, C4 and its 8-way
# shard, then the whole step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06v}
bash scripts/gpu_ab.sh $TAG rel rr2 rr3 || exit $?
timeout -k 10 300 python -u scripts/ab_variants.py run --step --config C4 --rounds 7 --reps 10 rel rr2 rr3 > gpurun_out/ab_${TAG}_step.txt 2>&1 || exit $?
grep -h '^{' gpurun_out/ab_${TAG}_step.txt
