#!/bin/bash
# Round 6: keyed sweep tiles of 16384 containers swept as two halves (one run and table row
# per 16384: the gather's segments twice as long) — the keyed tests, then A/B against the
# release tree's sweep (rel).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06w}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_keyed.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/ab_variants.py run --keyed --config C4 --rounds 7 --reps 10 rel st2 > gpurun_out/ab_${TAG}_keyed.txt 2>&1 || exit $?
grep -h '^{' gpurun_out/ab_${TAG}_keyed.txt
