#!/bin/bash
# The clamp in the fit: parity tests (both clamp modes), the C4 8-way rank emulated with the
# clamp in the fit and with the clamp correction, the default bench line.
#   bash scripts/gpu_r03v.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1
mkdir -p gpurun_out
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_$TAG.log
[ $rc -eq 0 ] || exit $rc
for W in 8 4; do
  for M in 1 0; do
    OUT=gpurun_out/emu_${TAG}_C4_w${W}_nc$M.json
    timeout -k 10 200 python3 -u bench.py --config C4 --scaling strong --emulate-world $W \
      --clamp-in-fit $M --no-cpu-baseline --no-keyed --no-pods --no-parse --no-dense \
      --steps 50 --warmup 5 > $OUT 2> ${OUT%.json}.err || exit $?
    echo "== C4 W=$W clamp_in_fit=$M: $(grep -o '"ms_per_step": [0-9.]*' $OUT)"
  done
done
timeout -k 10 240 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
grep -o '"ms_per_step": [0-9.]*' gpurun_out/bench_$TAG.json
