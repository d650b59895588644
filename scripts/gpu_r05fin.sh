#!/bin/bash
# Round 5 end (final tree): the round-end check (GPU suite, smoke, bench), then the
# rocprofv3 trace + PMC passes of the default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05fin}
bash scripts/gpu_final.sh $TAG || exit $?
bash scripts/profile.sh $TAG || exit $?
