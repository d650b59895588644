#!/bin/bash
# Round 5: the suite, rank 0's 8-way / 4-way C4 shard traced (per kernel), the 8-way
# shard's per-workgroup timeline, and whole-step A/Bs of the fit's claim / stream-length
# variants (8-way shard, one GPU).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05e}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_shard_trace.sh $TAG C4 8 4 || exit $?
timeout -k 10 200 python3 -u scripts/probe/timeline.py tl --config C4 --shard 8 --pipeline > gpurun_out/tl_${TAG}_c4w8.txt 2>&1 || exit $?
grep -v Warning gpurun_out/tl_${TAG}_c4w8.txt | grep -v "^ *ret\|^ *return\|amdgpu.ids" | tail -34
for SH in 8 1; do
  timeout -k 10 300 python3 -u scripts/ab_variants.py run --step --config C4 --shard $SH --rounds 7 --reps 20 base ngv qf2 qf4 qf4v \
    > gpurun_out/ab_${TAG}_step_s$SH.txt 2>&1 || exit $?
  grep '^{' gpurun_out/ab_${TAG}_step_s$SH.txt
done
