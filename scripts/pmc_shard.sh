#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one counter block each) of one rank's shard under strong
# scaling.  Usage (on the GPU box): bash scripts/pmc_shard.sh <tag> <config> <W>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; CFG=$2; W=$3
OUT=gpurun_out/pmcshard_${TAG}_${CFG}_w$W
mkdir -p $OUT
B="python3 bench.py --config $CFG --scaling strong --emulate-world $W --no-cpu-baseline --no-keyed --no-pods --no-parse --no-dense"
i=0
for pmc in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $pmc --output-format csv -d $OUT/pmc$i -o run \
    -- $B --steps 5 --warmup 1 > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i ($pmc) failed rc=$?"; exit 3; }
  echo "pmc $i ok: $pmc"
done
