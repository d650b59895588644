#!/bin/bash
# parity tests + traces + bench line, then an A/B of variants/ builds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
bash scripts/gpu_r03.sh $TAG || exit $?
bash scripts/gpu_ab.sh $TAG "$@" || exit $?
