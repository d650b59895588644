#!/bin/bash
# Round 5: node prep (clamp in the fit) behind the reduce's workgroups in one launch (base,
# the in-tree build) vs its own launch (npoff): the GPU tests that run the clamp in the fit
# first, then the step A/B at the C4 8-way / 4-way / 2-way ranks (identical totals checked).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05ab}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_shards_configs.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
for SH in 8 4 2; do
  timeout -k 10 300 python3 -u scripts/ab_variants.py run --step --config C4 --shard $SH --rounds 7 --reps 20 base npoff \
    > gpurun_out/ab_${TAG}_step_s$SH.txt 2>&1 || exit $?
  grep '^{' gpurun_out/ab_${TAG}_step_s$SH.txt
done
bash scripts/gpu_shard_trace.sh $TAG C4 8 || exit $?
