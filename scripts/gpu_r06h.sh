#!/bin/bash
# Round 6: the fit's workgroups in the node-prep reduce launch (fir; firlate = with the
# single-slot reduce tile loop, 5 waves per SIMD) against the release three-launch step,
# on the 8-way and 4-way C4 ranks (kcc_capacity_async, one process, interleaved)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06h}
mkdir -p gpurun_out
for W in 8 4; do
  timeout -k 10 300 python -u scripts/ab_variants.py run --step --config C4 --shard $W --rounds 7 --reps 20 fbase fir diag_firnf > gpurun_out/ab_${TAG}_w$W.txt 2>&1 || { echo "w$W rc=$?"; tail -5 gpurun_out/ab_${TAG}_w$W.txt; exit 1; }
  grep -h '^{' gpurun_out/ab_${TAG}_w$W.txt
done
