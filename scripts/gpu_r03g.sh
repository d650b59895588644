#!/bin/bash
# round-3 evidence: rocprofv3 trace + PMC passes of the default bench, then the
# strong-scaling emulation lines (rank 0's shard alone) for C4 and C5 at W = 2, 4, 8
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1
bash scripts/profile.sh $TAG || exit $?
bash scripts/gpu_emulate.sh $TAG C4 2 4 8 || exit $?
bash scripts/gpu_emulate.sh $TAG C5 1 2 4 8 || exit $?
