#!/bin/bash
# parity tests; C4 and C5 shard traces; strong-scaling emulation lines (W = 1, 2, 4, 8)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_shard_trace.sh $TAG C4 8 1 || exit $?
bash scripts/gpu_shard_trace.sh $TAG C5 8 || exit $?
bash scripts/gpu_emulate.sh $TAG C4 2 4 || exit $?
bash scripts/gpu_emulate.sh $TAG C5 2 4 || exit $?
