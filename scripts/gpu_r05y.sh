#!/bin/bash
# Round 5 end, part 2: rocprofv3 trace + PMC passes of the default bench (profiles/), then
# the keyed gather's LDS atomics measured: a timing build that sums records in a register.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05z}
bash scripts/profile.sh $TAG || exit $?
timeout -k 10 300 python3 -u scripts/ab_variants.py run --keyed --config C4 --rounds 5 --reps 10 base gnoat \
  > gpurun_out/ab_${TAG}_gnoat.txt 2>&1 || exit $?
grep '^{' gpurun_out/ab_${TAG}_gnoat.txt
