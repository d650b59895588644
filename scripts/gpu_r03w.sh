#!/bin/bash
# The clamp in the fit at 5.5 VALU: parity tests, the C4 2/4/8-way ranks (auto clamp mode)
# and rank 0's 8-way shard under rocprofv3, the default bench line.
#   bash scripts/gpu_r03w.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_emulate.sh $TAG C4 2 4 8 || exit $?
bash scripts/gpu_shard_trace.sh $TAG C4 8 || exit $?
timeout -k 10 240 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_$TAG.json
