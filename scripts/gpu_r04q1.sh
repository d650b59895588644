#!/bin/bash
# Round 4: the fit's first-claim cap at 1/16 and 1/32 of a workgroup's share (which also
# reaches C4's full-size fit) vs the release 1/8: bench lines at C4, alternating, 3 rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04q1}
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/variant_parity.py q1d16 q1d32 > gpurun_out/vp_$TAG.txt 2>&1 || exit $?
grep mismatches gpurun_out/vp_$TAG.txt
F="--no-cpu-baseline --no-keyed --no-pods --no-parse --no-dense"
for rep in 1 2 3; do
  for v in rel q1d16 q1d32; do
    L=""; [ $v != rel ] && L="--lib variants/libkcc_$v.so"
    timeout -k 10 200 python -u bench.py $F $L > gpurun_out/b_${TAG}_${v}_$rep.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/b_${TAG}_${v}_$rep.json'));print('C4 $v', round(d['ms_per_step'],5), 'fit', round(d['roofline_fit']['ms_per_launch'],5), d['totals_checksum'])"
  done
done
