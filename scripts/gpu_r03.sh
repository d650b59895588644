#!/bin/bash
# Round-3 check on the GPU box: parity tests, the default bench line, the C4 8-way shard
# trace.  Stops at the first failing step.
#   bash scripts/gpu_r03.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-x}
mkdir -p gpurun_out
bash scripts/gpu_round.sh $TAG || exit $?
timeout -k 10 240 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
cat gpurun_out/bench_$TAG.json
