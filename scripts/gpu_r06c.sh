#!/bin/bash
# Round 6: A/B of the reduce's forward per-item prefixes (adds) against the release walk-back
# (subtracts), C4 and its 8-way shard; then the bench line with the read flush.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06c}
bash scripts/gpu_ab.sh $TAG base fwd || exit $?
timeout -k 10 240 python -u bench.py --no-cpu-baseline --no-pods --no-parse > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
python3 -c "
import json
d = json.load(open('gpurun_out/bench_$TAG.json')); r = d['roofline_reduce']
print('step', d['ms_per_step'], 'red', r['ms_per_launch'], r['frac'], 'cold', r.get('ms_per_launch_cold'), r.get('frac_cold'), 'cold step', d['cold']['ms_per_step_median'], 'fit cold', d['cold']['fit_ms_per_launch'], d['roofline_valu']['ms_per_launch'])"
