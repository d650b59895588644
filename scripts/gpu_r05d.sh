#!/bin/bash
# Round 5: the suite, then rank 0's 8-way / 4-way C4 shard traced (per kernel) and the
# 8-way shard's per-workgroup timeline (KCC_TIMELINE variant).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05d}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_shard_trace.sh $TAG C4 8 4 || exit $?
timeout -k 10 200 python3 -u scripts/probe/timeline.py tl --config C4 --shard 8 --pipeline > gpurun_out/tl_${TAG}_c4w8.txt 2>&1 || exit $?
grep -v Warning gpurun_out/tl_${TAG}_c4w8.txt | grep -v "^ *ret\|^ *return\|amdgpu.ids" | tail -34
timeout -k 10 300 python3 -u scripts/ab_variants.py run --step --config C4 --shard 8 --rounds 7 --reps 20 base ngv \
  > gpurun_out/ab_${TAG}_ngv.txt 2>&1 || exit $?
grep '^{' gpurun_out/ab_${TAG}_ngv.txt
