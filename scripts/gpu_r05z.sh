#!/bin/bash
# Round 5 end, part 1: the round-end check (GPU suite, smoke, bench), then the strong-
# scaling emulation of C4 (W = 2, 4, 8) and C5 (W = 8).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05z}
bash scripts/gpu_final.sh $TAG || exit $?
bash scripts/gpu_emulate.sh $TAG C4 2 4 8 || exit $?
bash scripts/gpu_emulate.sh $TAG C5 8 || exit $?
