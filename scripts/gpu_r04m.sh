#!/bin/bash
# Round 4: keyed tests + A/B (balanced sweep tiles, reverse gather order, streaming record
# stores), per-kernel trace of the release keyed path.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04m}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_keyed.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_variants.py run --keyed --config C4 --rounds 5 --reps 10 base garev0 ntst kbold \
  > gpurun_out/ab_keyed_$TAG.txt 2>&1 || exit $?
grep '^{' gpurun_out/ab_keyed_$TAG.txt
K="python3 -u scripts/ab_variants.py run --keyed --config C4 --rounds 2 --reps 5 base"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kprof_$TAG -o run -- $K \
  > gpurun_out/kprof_${TAG}.log 2>&1 || exit $?
python3 scripts/kstats.py $(find gpurun_out/kprof_$TAG -name "*kernel_stats.csv") | grep -E "kb_|=="
