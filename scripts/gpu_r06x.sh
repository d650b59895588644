#!/bin/bash
# Round 6: per-kernel times of the keyed call, release sweep (rel) vs two-half sweep (st2)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06x}
mkdir -p gpurun_out
for v in ${VARS:-rel st2}; do
  OUT=gpurun_out/prof_${TAG}_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
    python3 -u scripts/ab_variants.py run --keyed --config C4 --rounds 3 --reps 10 $v > $OUT.log 2>&1 || exit $?
  python3 - <<PY
import csv, glob
for row in csv.DictReader(open(glob.glob('$OUT/*kernel_stats.csv')[0])):
    if 'kb_' in row['Name']:
        print('$v', row['Calls'], '%.2f us' % (float(row['AverageNs']) / 1e3), row['Name'][:50])
PY
done
