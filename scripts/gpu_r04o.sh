#!/bin/bash
# Round 4 strong-scaling emulation: rank 0's node shard of a W-way split timed alone
# (C4 W = 2, 4, 8; C5 with Zipf(1.2) pods per node, W = 8, 4, 2, 1) and the per-kernel
# rocprofv3 trace of C4's 8-way rank.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04o}
mkdir -p gpurun_out
bash scripts/gpu_emulate.sh $TAG C4 2 4 8 || exit $?
bash scripts/gpu_shard_trace.sh $TAG C4 8 || exit $?
for W in 8 4 2 1; do
  OUT=gpurun_out/emu_${TAG}_C5_w$W.json
  timeout -k 10 420 python3 -u bench.py --config C5 --scaling strong --emulate-world $W \
    --no-cpu-baseline --no-keyed --no-pods --no-parse --no-dense --steps 10 --warmup 2 \
    > $OUT 2> ${OUT%.json}.err || exit $?
  python3 -c "
import json;d=json.load(open('$OUT'))
print('C5 W=$W step', d['ms_per_step'], 'reduce', d['roofline_reduce']['ms_per_launch'], d['roofline_reduce']['frac'], 'fit', d['roofline_fit']['ms_per_launch'], 'valu', d['roofline_valu']['frac'], 'streamed', d['fit_stream']['fraction'], 'chk', d['totals_checksum'])"
done
