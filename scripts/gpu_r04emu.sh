#!/bin/bash
# Round 4 end: strong-scaling emulation of the round-end tree (C4 W = 2, 4, 8; C5 W = 8).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04e2}
bash scripts/gpu_emulate.sh $TAG C4 2 4 8 || exit $?
OUT=gpurun_out/emu_${TAG}_C5_w8.json
timeout -k 10 420 python3 -u bench.py --config C5 --scaling strong --emulate-world 8 \
  --no-cpu-baseline --no-keyed --no-pods --no-parse --no-dense --steps 10 --warmup 2 \
  > $OUT 2> ${OUT%.json}.err || exit $?
python3 -c "import json;d=json.load(open('$OUT'));print('C5 W=8', d['ms_per_step'], d['totals_checksum'])"
