#!/bin/bash
# Round 4: the keyed path's kernels (rocprofv3 trace + HBM bytes) on the release defaults.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04l}
mkdir -p gpurun_out
for v in s8 base; do
  K="python3 -u scripts/ab_variants.py run --keyed --config C4 --rounds 2 --reps 5 $v"
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kprof_$TAG/trace_$v -o run -- $K \
    > gpurun_out/kprof_${TAG}_$v.log 2>&1 || exit $?
  python3 scripts/kstats.py $(find gpurun_out/kprof_$TAG/trace_$v -name "*kernel_stats.csv")
  grep '^{' gpurun_out/kprof_${TAG}_$v.log
done
i=0
for pmc in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $pmc --output-format csv -d gpurun_out/kprof_$TAG/pmc$i -o run -- $K \
    > gpurun_out/kprof_${TAG}_pmc$i.log 2>&1 || { echo "pmc $pmc failed"; exit 3; }
  echo "pmc $pmc ok"
done
