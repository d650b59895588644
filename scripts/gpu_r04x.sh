#!/bin/bash
# Round 4: the fit reads its stream length once per workgroup (release) vs once per wave
# (ng0): fit parity tests, the 8-way timeline, bench lines at C4 and the 8-way rank.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04x}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -u scripts/probe/timeline.py tl --config C4 --shard 8 --pipeline > gpurun_out/tl_${TAG}_c4w8.txt 2>&1 || exit $?
grep -E "fit entry|spec records|fit loop|fit whole|fit segments" gpurun_out/tl_${TAG}_c4w8.txt
F="--no-cpu-baseline --no-keyed --no-pods --no-parse --no-dense"
for rep in 1 2; do
  for v in rel ngs0; do
    L=""; [ $v != rel ] && L="--lib variants/libkcc_$v.so"
    timeout -k 10 200 python -u bench.py $F $L --emulate-world 8 --steps 50 > gpurun_out/b_${TAG}_${v}_w8_$rep.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/b_${TAG}_${v}_w8_$rep.json'));print('C4/8 $v', round(d['ms_per_step'],5), 'fit', round(d['roofline_fit']['ms_per_launch'],5), d['totals_checksum'])"
    timeout -k 10 200 python -u bench.py $F $L > gpurun_out/b_${TAG}_${v}_$rep.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/b_${TAG}_${v}_$rep.json'));print('C4 $v', round(d['ms_per_step'],5), 'fit', round(d['roofline_fit']['ms_per_launch'],5), d['totals_checksum'])"
  done
done
