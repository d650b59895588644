#!/bin/bash
# parity tests, then the C4 / 8-way traces, then the timeline + A/B probe (one GPU call)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
bash scripts/gpu_round.sh $TAG || exit $?
bash scripts/gpu_probe.sh $TAG "$@"
