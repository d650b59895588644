#!/bin/bash
# Round 5: where the node-prep-in-reduce launch loses its time at the C4 8-way rank: the
# timing-only diagnostics (no wait on the reduce / plain node-sum stores; wrong totals
# expected for nosync) against base and the separate launch (npoff).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05ad}
mkdir -p gpurun_out
[ "${SKIP_TESTS:-0}" = 1 ] || timeout -k 10 700 python -u -m pytest tests/test_gpu_shards_configs.py tests/test_gpu_parity.py tests/test_faults_graphs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -20 gpurun_out/pytest_$TAG.log; exit 1; }
[ "${SKIP_TESTS:-0}" = 1 ] || tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 400 python3 -u scripts/ab_variants.py run --step --config C4 --shard 8 --rounds 7 --reps 20 \
  base ffin > gpurun_out/ab_${TAG}_step_s8.txt 2>&1 || exit $?
grep '^{' gpurun_out/ab_${TAG}_step_s8.txt
timeout -k 10 300 python3 -u scripts/ab_variants.py run --step --config C4 --shard 4 --rounds 7 --reps 20 \
  base ffin > gpurun_out/ab_${TAG}_step_s4.txt 2>&1 || exit $?
grep '^{' gpurun_out/ab_${TAG}_step_s4.txt
timeout -k 10 300 python3 -u scripts/ab_variants.py run --step --config C4 --shard 1 --rounds 5 --reps 10 \
  base ffin > gpurun_out/ab_${TAG}_step_s1.txt 2>&1 || exit $?
grep '^{' gpurun_out/ab_${TAG}_step_s1.txt
