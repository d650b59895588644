#!/bin/bash
# Round 5: the whole -m gpu suite (new: C1 end to end, C5 whole cluster, cross-rank fault
# marks, the in-library all-reduce check), then the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05b}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  --durations=15 > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
python3 -c "
import json;d=json.load(open('gpurun_out/bench_$TAG.json'))
print('step', d['ms_per_step'], 'reduce', d['roofline_reduce']['ms_per_launch'], d['roofline_reduce']['frac'], 'fit', d['roofline_fit']['ms_per_launch'], 'valu', d['roofline_valu']['frac'], 'keyed', d['keyed']['ms_per_launch'], d['keyed']['roofline']['frac'], 'chk', d['totals_checksum'])"
