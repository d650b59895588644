#!/bin/bash
# Round 5: per-kernel times of the keyed path, 6-byte records (base) vs round 4's (prev).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05m}
mkdir -p gpurun_out
for V in prev base; do
  OUT=gpurun_out/kprof_${TAG}_$V
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run \
    -- python3 scripts/ab_variants.py run --keyed --config C4 --rounds 2 --reps 5 $V > $OUT/ab.log 2>&1 || exit $?
  f=$(find $OUT -name "*kernel_stats.csv" | head -1)
  echo "== $V"
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'kb_' in r['Name']:
        print(f"  {r['Name'][:60]:60s} calls={r['Calls']:>5} avg_us={float(r['AverageNs'])/1e3:8.2f}")
PY
done
