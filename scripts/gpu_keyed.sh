#!/bin/bash
# Keyed (list-order) reduce on the GPU: its tests, then the bench's keyed leg under a
# rocprofv3 kernel trace.  Usage (on the GPU box): bash scripts/gpu_keyed.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-keyed}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_keyed.py -m gpu -v --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_keyed.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -12 gpurun_out/pytest_keyed.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run \
  -- python3 bench.py --no-parse --no-cpu-baseline > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"
exit $rc
