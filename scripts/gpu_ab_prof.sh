#!/bin/bash
# Guarded GPU session: parity tests, A/B of the variants/ builds named in $@ (fit =
# node_prep + fit + clamp_apply), then a rocprofv3 kernel trace of each variant alone.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 540 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_variants.py run "$@" > gpurun_out/ab.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/ab.log | tail -8
[ $rc -eq 0 ] || exit $rc
for v in "$@"; do
  case $v in --*) continue;; esac
  timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_$v -o run \
    -- python3 scripts/ab_variants.py run --rounds 2 $v > gpurun_out/ab_$v.log 2>&1 || exit $?
done
echo "prof ok"
