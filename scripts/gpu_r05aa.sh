#!/bin/bash
# Round 5: the fit's claims sized by the workgroup's rate against its segment's (ad), and
# with a 4-group static first claim (adq), vs base; step A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05aa}
mkdir -p gpurun_out
for SH in 1 8 4 2; do
  timeout -k 10 300 python3 -u scripts/ab_variants.py run --step --config C4 --shard $SH --rounds 7 --reps 20 base ad adq \
    > gpurun_out/ab_${TAG}_step_s$SH.txt 2>&1 || exit $?
  grep '^{' gpurun_out/ab_${TAG}_step_s$SH.txt
done
