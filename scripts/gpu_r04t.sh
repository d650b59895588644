#!/bin/bash
# Round 4: the spec ranks' workgroups behind the reduce's (release) vs in front (rk0): the
# whole -m gpu suite on the release build, then bench lines at C4 and rank 0 of an 8-way
# split, alternating, twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04t}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
F="--no-cpu-baseline --no-keyed --no-pods --no-parse --no-dense"
for rep in 1 2 3; do
  for v in rel rk0; do
    L=""; [ $v != rel ] && L="--lib variants/libkcc_$v.so"
    timeout -k 10 200 python -u bench.py $F $L > gpurun_out/b_${TAG}_${v}_$rep.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/b_${TAG}_${v}_$rep.json'));print('C4 $v', round(d['ms_per_step'],5), 'reduce', round(d['roofline_reduce']['ms_per_launch'],5), round(d['roofline_reduce']['frac'],4), d['totals_checksum'])"
  done
done
for rep in 1 2; do
  for v in rel rk0; do
    L=""; [ $v != rel ] && L="--lib variants/libkcc_$v.so"
    timeout -k 10 200 python -u bench.py $F $L --emulate-world 8 --steps 50 > gpurun_out/b_${TAG}_${v}_w8_$rep.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/b_${TAG}_${v}_w8_$rep.json'));print('C4/8 $v', round(d['ms_per_step'],5), 'reduce', round(d['roofline_reduce']['ms_per_launch'],5), d['totals_checksum'])"
  done
done
