#!/bin/bash
# Round 5: the 8-way / 4-way C4 rank step's kernels and the idle gaps between them
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05ah}
bash scripts/gpu_shard_trace.sh $TAG C4 8 4 || exit $?
for W in 8 4; do
  f=$(find gpurun_out/shard_${TAG}_C4_w$W -name "*kernel_trace.csv" | head -1)
  echo "== W=$W"; python3 scripts/trace_gaps.py "$f" reduce_kernel || exit $?
done
