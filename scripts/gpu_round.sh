#!/bin/bash
# One guarded GPU session: parity tests, then kernel traces of the C4 step on one GPU and
# of rank 0's 8-way shard.  Stops at any abort, signal or time limit.
#   bash scripts/gpu_round.sh <tag> [pytest -k expr]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-x}
K=${2:-}
mkdir -p gpurun_out
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread \
  "${KARG[@]}" > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_shard_trace.sh $TAG C4 8 1
