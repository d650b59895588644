#!/bin/bash
# Round 5 end, second pass (node prep in the reduce launch): the round-end check (GPU suite,
# smoke, bench), the strong-scaling rank emulations of C4 and C5, then the rocprofv3 trace
# + PMC passes of the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05fin2}
bash scripts/gpu_final.sh $TAG || exit $?
bash scripts/gpu_emulate.sh $TAG C4 8 4 2 || exit $?
bash scripts/gpu_emulate.sh $TAG C5 8 || exit $?
bash scripts/profile.sh $TAG || exit $?
