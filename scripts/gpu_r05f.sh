#!/bin/bash
# Round 5: the fit's static share vs the claim queue (whole step A/B at the C4 8-way /
# 4-way shards and C4), the reduce's strip layout A/B, the static build's 8-way timeline,
# the 8-way trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05f}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_shards_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_shard_trace.sh $TAG C4 8 || exit $?
for SH in 8 4 1; do
  timeout -k 10 300 python3 -u scripts/ab_variants.py run --step --config C4 --shard $SH --rounds 7 --reps 20 base fst stt \
    > gpurun_out/ab_${TAG}_step_s$SH.txt 2>&1 || exit $?
  grep '^{' gpurun_out/ab_${TAG}_step_s$SH.txt
done
for SH in 1 8; do
  timeout -k 10 300 python3 -u scripts/ab_variants.py run --config C4 --shard $SH --rounds 7 --reps 20 base stt \
    > gpurun_out/ab_${TAG}_red_s$SH.txt 2>&1 || exit $?
  grep '^{' gpurun_out/ab_${TAG}_red_s$SH.txt
done
timeout -k 10 200 python3 -u scripts/probe/timeline.py fsttl --config C4 --shard 8 --pipeline > gpurun_out/tl_${TAG}_fst_c4w8.txt 2>&1 || exit $?
grep -v Warning gpurun_out/tl_${TAG}_fst_c4w8.txt | grep -v "^ *ret\|^ *return\|amdgpu.ids" | grep "fit\|reduce waves"
