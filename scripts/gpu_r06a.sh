#!/bin/bash
# Round 6, first pass: the round-end check (GPU suite incl. the new inlib / ISA cases, smoke,
# the default bench line with its cold-cache leg), then the 8-way C4 rank emulation.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06a}
bash scripts/gpu_final.sh $TAG || exit $?
bash scripts/gpu_emulate.sh $TAG C4 8 || exit $?
python3 -c "
import json
for f in ['gpurun_out/bench_$TAG.json', 'gpurun_out/emu_${TAG}_C4_w8.json']:
    d = json.load(open(f)); r = d['roofline_reduce']
    print(f, 'step', d['ms_per_step'], 'red', r['ms_per_launch'], r['frac'], 'cold', r.get('ms_per_launch_cold'), r.get('frac_cold'), 'cold step', d['cold']['ms_per_step_median'])"
