#!/bin/bash
# Round 5: the clamp in the fit (now with node prep in the reduce launch) on the 2-way C4
# rank (2.05e9 node rows x specs, above the 1.1e9 threshold) against clamp_apply
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05ar}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u scripts/ab_variants.py run --step --config C4 --shard 2 --rounds 11 --reps 20 \
  base cif3 base2 > gpurun_out/ab_${TAG}_step_s2.txt 2>&1 || exit $?
grep '^{' gpurun_out/ab_${TAG}_step_s2.txt
