#!/bin/bash
# rocprofv3 kernel traces of one rank's shard under strong scaling (C4: 1M nodes split
# over W ranks), W = each argument.  Usage (on the GPU box):
#   bash scripts/gpu_shard_trace.sh <tag> <config> <W>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; CFG=$2; shift 2
mkdir -p gpurun_out
for W in "$@"; do
  OUT=gpurun_out/shard_${TAG}_${CFG}_w$W
  mkdir -p $OUT
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run \
    -- python3 bench.py --config $CFG --scaling strong --emulate-world $W --no-cpu-baseline \
       --no-keyed --no-pods --no-parse --no-dense --steps 50 --warmup 5 > $OUT/bench.log 2>&1 || exit $?
  f=$(find $OUT -name "*kernel_stats.csv" | head -1)
  echo "== $CFG W=$W: $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench.log)"
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"  {r['Name'][:44]:44s} calls={r['Calls']:>5} avg_us={float(r['AverageNs'])/1e3:8.2f}")
PY
done
