#!/bin/bash
# Round 5: does the kernel-argument placement explain the workgroups' late starts?
# The 8-way C4 timeline and the whole-step A/B under HIP_FORCE_DEV_KERNARG=0 and =1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05i}
mkdir -p gpurun_out
for KA in 0 1; do
  HIP_FORCE_DEV_KERNARG=$KA timeout -k 10 200 python3 -u scripts/probe/timeline.py tl --config C4 --shard 8 --pipeline \
    > gpurun_out/tl_${TAG}_ka$KA.txt 2>&1 || exit $?
  echo "== HIP_FORCE_DEV_KERNARG=$KA"
  grep -v Warning gpurun_out/tl_${TAG}_ka$KA.txt | grep "fit entry\|spec records\|fit loop\|fit whole\|reduce waves\|node_prep whole"
  for SH in 8 1; do
    HIP_FORCE_DEV_KERNARG=$KA timeout -k 10 300 python3 -u scripts/ab_variants.py run --step --config C4 --shard $SH --rounds 5 --reps 20 base nofuse \
      > gpurun_out/ab_${TAG}_ka${KA}_s$SH.txt 2>&1 || exit $?
    grep '^{' gpurun_out/ab_${TAG}_ka${KA}_s$SH.txt
  done
done
