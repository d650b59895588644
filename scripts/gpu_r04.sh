#!/bin/bash
# Round-4 GPU session: the new fault / graph / exchange-check tests first, then the whole
# -m gpu suite, an A/B of variants/ builds (optional) and the default bench line.
#   bash scripts/gpu_r04.sh <tag> [variant ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-x}; shift
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_faults_graphs.py tests/test_shard_gloo.py \
  tests/test_gpu_shards_configs.py -k "fault or graph or efault or exchange or bench" -m gpu -x -v \
  --timeout 150 --timeout-method thread > gpurun_out/pytest_new_$TAG.log 2>&1
rc=$?; echo "new tests rc=$rc"; tail -5 gpurun_out/pytest_new_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
if [ $# -gt 0 ]; then
  bash scripts/gpu_ab.sh $TAG "$@" || exit $?
fi
timeout -k 10 240 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
python3 -c "
import json;d=json.load(open('gpurun_out/bench_$TAG.json'))
print('step', d['ms_per_step'], 'reduce', d['roofline_reduce']['ms_per_launch'], d['roofline_reduce']['frac'], 'fit', d['roofline_fit']['ms_per_launch'], 'keyed', d['keyed']['ms_per_launch'], d['keyed']['roofline']['frac'], 'chk', d['totals_checksum'])"
# C5 (Zipf(1.2) pods per node) strong-scaling emulation: rank 0's shard of 8, then all of C5
if [ "${C5:-0}" = 1 ]; then
  for W in 8 1; do
    OUT=gpurun_out/emu_${TAG}_C5_w$W.json
    timeout -k 10 420 python3 -u bench.py --config C5 --scaling strong --emulate-world $W \
      --no-cpu-baseline --no-keyed --no-pods --no-parse --no-dense --steps 10 --warmup 2 \
      > $OUT 2> ${OUT%.json}.err || exit $?
    python3 -c "
import json;d=json.load(open('$OUT'))
print('C5 W=$W step', d['ms_per_step'], 'reduce', d['roofline_reduce']['ms_per_launch'], 'fit', d['roofline_fit']['ms_per_launch'], 'valu', d['roofline_valu']['frac'], 'streamed', d['fit_stream']['fraction'], 'containers', d['config']['containers_rank0'])"
  done
fi
