#!/bin/bash
# Parse row on the GPU: its tests, smoke, then the bench (with the parse leg) under a
# rocprofv3 kernel trace.  Usage (on the GPU box): bash scripts/gpu_parse.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-parse}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parse.py -m gpu -v --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_parse.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -12 gpurun_out/pytest_parse.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run \
  -- python3 bench.py > gpurun_out/bench_$TAG.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_$TAG.log
exit $rc
