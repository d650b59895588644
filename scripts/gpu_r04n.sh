#!/bin/bash
# Round 4 release measurements: the whole -m gpu suite, the quantity-parse A/B (streaming
# stores, register path v1), the default bench line, the rocprofv3 trace + PMC passes of
# the bench (profiles/), and the shards' HBM bytes (C4 W=2/4/8, C5 W=8).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04n}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_variants.py run --parse --config C4 --rounds 5 --reps 10 base pnt0 pqv1 \
  > gpurun_out/ab_parse_$TAG.txt 2>&1 || exit $?
grep '^{' gpurun_out/ab_parse_$TAG.txt
timeout -k 10 240 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
python3 -c "
import json;d=json.load(open('gpurun_out/bench_$TAG.json'))
print('step', d['ms_per_step'], 'reduce', d['roofline_reduce']['ms_per_launch'], d['roofline_reduce']['frac'], 'fit', d['roofline_fit']['ms_per_launch'], 'valu', d['roofline_valu']['frac'], 'keyed', d['keyed']['ms_per_launch'], d['keyed']['roofline']['frac'], 'qty', d['parse']['quantity']['ms_per_launch'], 'chk', d['totals_checksum'])"
bash scripts/profile.sh $TAG || exit $?
bash scripts/gpu_pmc_shards.sh $TAG || exit $?
