#!/bin/bash
# Round 5 baseline on this round's box: the -m gpu suite, the default bench line, and
# rocprofv3 per-kernel traces of the C4 step at W = 1 and of rank 0's 8-way shard.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05a}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
python3 -c "
import json;d=json.load(open('gpurun_out/bench_$TAG.json'))
print('step', d['ms_per_step'], 'reduce', d['roofline_reduce']['ms_per_launch'], d['roofline_reduce']['frac'], 'fit', d['roofline_fit']['ms_per_launch'], 'valu', d['roofline_valu']['frac'], 'keyed', d['keyed']['ms_per_launch'], d['keyed']['roofline']['frac'], 'chk', d['totals_checksum'])"
bash scripts/gpu_shard_trace.sh $TAG C4 8 1 || exit $?
