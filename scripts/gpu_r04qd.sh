#!/bin/bash
# Round 4: guided-claim divisor 3 / 4 (release 2) and first-claim cap 1/4 (release 1/8):
# variant parity, then bench lines at the 8-way C4 rank and C4, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04qd}
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/variant_parity.py qdiv3 qdiv4 q1d4b > gpurun_out/vp_$TAG.txt 2>&1 || exit $?
grep mismatches gpurun_out/vp_$TAG.txt
F="--no-cpu-baseline --no-keyed --no-pods --no-parse --no-dense"
for rep in 1 2; do
  for v in rel qdiv3 qdiv4 q1d4b; do
    L=""; [ $v != rel ] && L="--lib variants/libkcc_$v.so"
    timeout -k 10 200 python -u bench.py $F $L --emulate-world 8 --steps 50 > gpurun_out/b_${TAG}_${v}_w8_$rep.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/b_${TAG}_${v}_w8_$rep.json'));print('C4/8 $v', round(d['ms_per_step'],5), 'fit', round(d['roofline_fit']['ms_per_launch'],5), d['totals_checksum'])"
  done
done
for v in rel qdiv3 qdiv4; do
  L=""; [ $v != rel ] && L="--lib variants/libkcc_$v.so"
  timeout -k 10 200 python -u bench.py $F $L > gpurun_out/b_${TAG}_${v}.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/b_${TAG}_${v}.json'));print('C4 $v', round(d['ms_per_step'],5), 'fit', round(d['roofline_fit']['ms_per_launch'],5), d['totals_checksum'])"
done
