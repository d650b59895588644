#!/bin/bash
# parity tests (incl. the p2p exchange between processes sharing the GPU), then the
# multi-rank bench rehearsal (2 gloo ranks, p2p exchange) for C3 and C4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_multirank.sh C3 > gpurun_out/mr_${TAG}_c3.txt 2>&1 || { cat gpurun_out/mr_${TAG}_c3.txt; exit 3; }
cat gpurun_out/mr_${TAG}_c3.txt
bash scripts/gpu_multirank.sh C4 > gpurun_out/mr_${TAG}_c4.txt 2>&1 || { cat gpurun_out/mr_${TAG}_c4.txt; exit 3; }
cat gpurun_out/mr_${TAG}_c4.txt
