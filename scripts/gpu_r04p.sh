#!/bin/bash
# Round 4: the clamp correction beside the fit (KCC_CLAMP_CONCURRENT): the whole -m gpu
# suite on it, then bench lines release vs -DKCC_CLAMP_CONCURRENT=0 at C4 and rank 0 of an
# 8-way split (both clamp modes there), and the per-kernel trace of the C4 step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04p}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
F="--no-cpu-baseline --no-keyed --no-pods --no-parse --no-dense"
for rep in 1 2; do
  for v in rel cc0; do
    L=""; [ $v = cc0 ] && L="--lib variants/libkcc_cc0.so"
    timeout -k 10 200 python -u bench.py $F $L > gpurun_out/b_${TAG}_${v}_$rep.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/b_${TAG}_${v}_$rep.json'));print('C4 $v', d['ms_per_step'], d['totals_checksum'])"
  done
done
for v in rel cc0; do
  L=""; [ $v = cc0 ] && L="--lib variants/libkcc_cc0.so"
  for m in 0 1; do
    timeout -k 10 200 python -u bench.py $F $L --emulate-world 8 --steps 50 --clamp-in-fit $m > gpurun_out/b_${TAG}_${v}_w8m$m.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/b_${TAG}_${v}_w8m$m.json'));print('C4/8 $v clamp_in_fit=$m', d['ms_per_step'], d['totals_checksum'])"
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py $F --steps 20 \
  > gpurun_out/prof_$TAG.log 2>&1 || exit $?
python3 scripts/kstats.py $(find gpurun_out/prof_$TAG -name "*kernel_stats.csv") | head -8
