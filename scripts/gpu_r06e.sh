#!/bin/bash
# Round 6: keyed-gather variants (nt loads, 12-segment sub-batches, no-atomics timing builds)
# against round 5's gather, then the default bench line (read-flush cold leg).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06e}
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/ab_variants.py run --keyed --config C4 --rounds 7 --reps 10 gold ga0 gant gau12 ganoatom goldnoatom > gpurun_out/ab_${TAG}_keyed.txt 2>&1 || exit $?
grep -h '^{' gpurun_out/ab_${TAG}_keyed.txt
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
python3 -c "
import json
d = json.load(open('gpurun_out/bench_$TAG.json')); r = d['roofline_reduce']
print('step', d['ms_per_step'], 'red', r['ms_per_launch'], r['frac'], 'cold', r.get('ms_per_launch_cold'), r.get('frac_cold'), 'cold step', d['cold']['ms_per_step_median'], 'fit cold', d['cold']['fit_ms_per_launch'], d['roofline_valu']['ms_per_launch'], 'keyed', d['keyed']['ms_per_launch'], d['keyed']['roofline']['frac'], d['keyed']['equals_csr_reduce'])"
