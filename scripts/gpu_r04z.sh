#!/bin/bash
# Round 4: the fit's static first claim capped at share / Q1_DIV (q1d2, q1d4, q1d8) vs qsz
# (release): parity on each variant's library (GPU parity subset), bench lines at the 8-way
# rank and C4, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04z}
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/variant_parity.py q1d2 q1d4 q1d8 > gpurun_out/vp_$TAG.txt 2>&1; echo "variant parity rc=$?"; tail -3 gpurun_out/vp_$TAG.txt
F="--no-cpu-baseline --no-keyed --no-pods --no-parse --no-dense"
for rep in 1 2; do
  for v in rel q1d2 q1d4 q1d8; do
    L=""; [ $v != rel ] && L="--lib variants/libkcc_$v.so"
    timeout -k 10 200 python -u bench.py $F $L --emulate-world 8 --steps 50 > gpurun_out/b_${TAG}_${v}_w8_$rep.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/b_${TAG}_${v}_w8_$rep.json'));print('C4/8 $v', round(d['ms_per_step'],5), 'fit', round(d['roofline_fit']['ms_per_launch'],5), d['totals_checksum'])"
  done
done
for v in rel q1d4; do
  L=""; [ $v != rel ] && L="--lib variants/libkcc_$v.so"
  timeout -k 10 200 python -u bench.py $F $L > gpurun_out/b_${TAG}_${v}.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/b_${TAG}_${v}.json'));print('C4 $v', round(d['ms_per_step'],5), 'fit', round(d['roofline_fit']['ms_per_launch'],5), d['totals_checksum'])"
done
