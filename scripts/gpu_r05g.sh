#!/bin/bash
# Round 5: the fit's fused finalize with relaxed arrivals (base) vs a fit_finalize launch
# (nofuse), whole-step A/B at the C4 8-way / 4-way shards and C4; the keyed reduce's
# pipelined persistent sweep (kswp) vs base; the full GPU suite first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05g}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
for SH in 8 4 1; do
  timeout -k 10 300 python3 -u scripts/ab_variants.py run --step --config C4 --shard $SH --rounds 7 --reps 20 base nofuse \
    > gpurun_out/ab_${TAG}_step_s$SH.txt 2>&1 || exit $?
  grep '^{' gpurun_out/ab_${TAG}_step_s$SH.txt
done
timeout -k 10 300 python3 -u scripts/ab_variants.py run --keyed --config C4 --rounds 7 --reps 10 base kswp \
  > gpurun_out/ab_${TAG}_keyed.txt 2>&1 || exit $?
grep '^{' gpurun_out/ab_${TAG}_keyed.txt
bash scripts/gpu_shard_trace.sh $TAG C4 8 || exit $?
