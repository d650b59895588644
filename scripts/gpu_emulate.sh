#!/bin/bash
# Strong-scaling emulation on one GPU: rank 0's node shard of a W-way split, timed alone
# (no all-reduce: that exchange needs W devices), for each config and W given.
#   bash scripts/gpu_emulate.sh <tag> <config> <W>...
# -> gpurun_out/emu_<tag>_<config>_w<W>.json (one bench line each); EXTRA: more bench flags
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; CFG=$2; shift 2
mkdir -p gpurun_out
for W in "$@"; do
  OUT=gpurun_out/emu_${TAG}_${CFG}_w$W.json
  timeout -k 10 200 python3 -u bench.py --config $CFG --scaling strong --emulate-world $W \
    --no-cpu-baseline --no-keyed --no-pods --no-parse --no-dense --steps 50 --warmup 5 ${EXTRA:-} \
    > $OUT 2> ${OUT%.json}.err || exit $?
  echo "== $CFG W=$W: $(grep -o '"ms_per_step": [0-9.]*' $OUT)"
done
