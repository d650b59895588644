#!/bin/bash
# Round 6 close: the committed tree's GPU suite, smoke(), the default bench line, the 8-way
# rank (emulated), and a rocprofv3 kernel trace of that rank (VERDICT r5 item 1's trace).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06n}
bash scripts/gpu_final.sh $TAG || exit $?
bash scripts/gpu_emulate.sh $TAG C4 8 || exit $?
OUT=gpurun_out/prof_${TAG}_w8; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --config C4 --scaling strong --emulate-world 8 --no-cpu-baseline --no-keyed \
  --no-pods --no-parse --no-dense --steps 50 --warmup 5 > $OUT/trace.log 2>&1 || exit $?
python3 - <<PY
import csv, glob
for row in csv.DictReader(open(glob.glob('$OUT/trace/*kernel_stats.csv')[0])):
    print('rocprof w8', row['Calls'], '%.2f us' % (float(row['AverageNs']) / 1e3), row['Name'][:60])
PY
