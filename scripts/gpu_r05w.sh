#!/bin/bash
# Round 5: the keyed gather over bucket pairs with parts by CU count (base) vs one bucket
# per workgroup (bpg1): keyed GPU tests, A/B at C4, per-kernel times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05w}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_keyed.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u scripts/ab_variants.py run --keyed --config C4 --rounds 9 --reps 10 rel base \
  > gpurun_out/ab_${TAG}_keyed.txt 2>&1 || exit $?
grep '^{' gpurun_out/ab_${TAG}_keyed.txt
for V in rel base; do
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
