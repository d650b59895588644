#!/bin/bash
# Round 4 end: the round-end check (GPU suite, smoke, bench), then the 8-way C4 rank with
# the first-claim cap at 1/8 (release), 1/16 and off, alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04fin}
bash scripts/gpu_final.sh $TAG || exit $?
F="--no-cpu-baseline --no-keyed --no-pods --no-parse --no-dense"
for rep in 1 2; do
  for v in rel q1d16 q1d0; do
    L=""; [ $v != rel ] && L="--lib variants/libkcc_$v.so"
    timeout -k 10 200 python -u bench.py $F $L --emulate-world 8 --steps 50 > gpurun_out/b_${TAG}_${v}_w8_$rep.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/b_${TAG}_${v}_w8_$rep.json'));print('C4/8 $v', round(d['ms_per_step'],5), 'fit', round(d['roofline_fit']['ms_per_launch'],5), d['totals_checksum'])"
  done
done
