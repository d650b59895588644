#!/bin/bash
# Round 5: the keyed sweep's 6-byte records (base, u24: 24 gather segments per wave in
# flight) vs round 4's 8-byte records with the pipelined sweep (prev): keyed GPU tests,
# then the A/B at C4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05l}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_keyed.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u scripts/ab_variants.py run --keyed --config C4 --rounds 7 --reps 10 prev base u24 u32 \
  > gpurun_out/ab_${TAG}_keyed.txt 2>&1 || exit $?
grep '^{' gpurun_out/ab_${TAG}_keyed.txt
