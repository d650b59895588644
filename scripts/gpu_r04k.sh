#!/bin/bash
# Round 4: the whole -m gpu suite on the release defaults, the keyed and quantity-parse
# A/Bs, the default bench line, the HIP-graph bench line, rank 0 of an 8-way C4 split
# (eager and graph).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04k}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_variants.py run --keyed --config C4 --rounds 5 --reps 10 base kbold s16u8p1 s16u16p1 s8u8p1 s8u16p1 \
  > gpurun_out/ab_keyed_$TAG.txt 2>&1 || exit $?
grep '^{' gpurun_out/ab_keyed_$TAG.txt
timeout -k 10 300 python -u scripts/ab_variants.py run --parse --config C4 --rounds 5 --reps 10 base pqv1 \
  > gpurun_out/ab_parse_$TAG.txt 2>&1 || exit $?
grep '^{' gpurun_out/ab_parse_$TAG.txt
timeout -k 10 240 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
python3 -c "
import json;d=json.load(open('gpurun_out/bench_$TAG.json'))
print('step', d['ms_per_step'], 'reduce', d['roofline_reduce']['ms_per_launch'], d['roofline_reduce']['frac'], 'fit', d['roofline_fit']['ms_per_launch'], 'valu', d['roofline_valu']['frac'], 'keyed', d['keyed']['ms_per_launch'], d['keyed']['roofline']['frac'], 'qty', d['parse']['quantity']['ms_per_launch'] if 'quantity' in d.get('parse', {}) else None, 'chk', d['totals_checksum'])"
timeout -k 10 240 python -u bench.py --graph 1 --no-cpu-baseline --no-keyed --no-pods --no-parse --no-dense \
  > gpurun_out/bench_${TAG}_graph.json 2> gpurun_out/bench_${TAG}_graph.err || exit $?
python3 -c "import json;d=json.load(open('gpurun_out/bench_${TAG}_graph.json'));print('graph step', d['ms_per_step'], 'chk', d['totals_checksum'])"
bash scripts/gpu_emulate.sh ${TAG} C4 8 || exit $?
EXTRA="--graph 1" bash scripts/gpu_emulate.sh ${TAG}g C4 8 || exit $?
