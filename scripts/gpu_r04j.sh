#!/bin/bash
# Round 4: the memory-bound skip A/B with per-kernel rocprofv3 stats of each variant (the
# fit step = node_prep + fit + clamp correction), the keyed A/B, bench lines (eager and
# HIP-graph replay), rank 0 of an 8-way C4 split.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04j}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parse.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh $TAG base msk0 || exit $?
for v in base msk0; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_$v -o run \
    -- python3 -u scripts/ab_variants.py run --config C4 --rounds 2 --reps 10 $v \
    > gpurun_out/prof_${TAG}_$v.log 2>&1 || exit $?
  python3 scripts/kstats.py $(find gpurun_out/prof_${TAG}_$v -name "*kernel_stats.csv") || true
done
timeout -k 10 300 python -u scripts/ab_variants.py run --keyed --config C4 --rounds 5 --reps 10 kbold s16u8 s16u8p1 s16u16p1 s8u8p1 s8u16p1 \
  > gpurun_out/ab_keyed_$TAG.txt 2>&1 || exit $?
grep '^{' gpurun_out/ab_keyed_$TAG.txt
timeout -k 10 240 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
python3 -c "
import json;d=json.load(open('gpurun_out/bench_$TAG.json'))
v=d['roofline_valu']
print('step', d['ms_per_step'], 'reduce', d['roofline_reduce']['ms_per_launch'], d['roofline_reduce']['frac'], 'fit', d['roofline_fit']['ms_per_launch'], 'valu', v['frac'], 'mskip', v.get('mskip_fraction'), 'keyed', d['keyed']['ms_per_launch'], d['keyed']['roofline']['frac'], 'chk', d['totals_checksum'])"
timeout -k 10 240 python -u bench.py --graph 1 --no-cpu-baseline --no-keyed --no-pods --no-parse --no-dense \
  > gpurun_out/bench_${TAG}_graph.json 2> gpurun_out/bench_${TAG}_graph.err || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_graph.json'));print('graph step', d['ms_per_step'], 'chk', d['totals_checksum'])"
bash scripts/gpu_emulate.sh ${TAG} C4 8 || exit $?
EXTRA="--graph 1" bash scripts/gpu_emulate.sh ${TAG}g C4 8 || exit $?
timeout -k 10 300 python -u scripts/ab_variants.py run --parse --config C4 --rounds 5 --reps 10 base pqv1 \
  > gpurun_out/ab_parse_$TAG.txt 2>&1 || exit $?
grep '^{' gpurun_out/ab_parse_$TAG.txt
