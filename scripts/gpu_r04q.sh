#!/bin/bash
# Round 4: the clamp correction beside the fit, queued before (cc1) or after (cc2) the fit,
# against the release order (after the fit): parity of both variants on the clamp tests,
# then bench lines at C4 and rank 0 of an 8-way split (clamp-correction mode).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04q}
mkdir -p gpurun_out
F="--no-cpu-baseline --no-keyed --no-pods --no-parse --no-dense"
for rep in 1 2; do
  for v in rel cc2 cc1; do
    L=""; [ $v != rel ] && L="--lib variants/libkcc_$v.so"
    timeout -k 10 200 python -u bench.py $F $L > gpurun_out/b_${TAG}_${v}_$rep.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/b_${TAG}_${v}_$rep.json'));print('C4 $v', d['ms_per_step'], d['totals_checksum'])"
  done
done
for v in rel cc2; do
  L=""; [ $v != rel ] && L="--lib variants/libkcc_$v.so"
  timeout -k 10 200 python -u bench.py $F $L --emulate-world 8 --steps 50 --clamp-in-fit 0 > gpurun_out/b_${TAG}_${v}_w8m0.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/b_${TAG}_${v}_w8m0.json'));print('C4/8 $v clamp_in_fit=0', d['ms_per_step'], d['totals_checksum'])"
done
