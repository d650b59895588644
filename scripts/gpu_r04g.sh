#!/bin/bash
# Keyed one-sweep path: its tests, an A/B against the 4-kernel path and gather splits, and
# the bench's keyed leg under a kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04g}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_keyed.py -m gpu -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_keyed_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_keyed_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_variants.py run --keyed --config C4 --rounds 5 --reps 10 kbold s16u8 s16u8p1 s16u16p1 s8u8p1 s8u16p1 \
  > gpurun_out/ab_keyed_$TAG.txt 2>&1 || exit $?
grep '^{' gpurun_out/ab_keyed_$TAG.txt
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_keyed_$TAG -o run \
  -- python3 bench.py --no-parse --no-cpu-baseline --no-pods --no-dense > gpurun_out/bench_keyed_$TAG.log 2>&1 || exit $?
f=$(find gpurun_out/prof_keyed_$TAG -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"  {r['Name'][:44]:44s} calls={r['Calls']:>5} avg_us={float(r['AverageNs'])/1e3:8.2f}")
PY
