#!/bin/bash
# Round 6: per-kernel timing from the dispatch packets (hipExtLaunchKernel events): the GPU
# suite, smoke(), the default bench line, the same with the kernel events inside the timed
# steps, the 8-way rank, and a rocprofv3 kernel trace to compare the averages with.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06m}
bash scripts/gpu_final.sh $TAG || exit $?
timeout -k 10 240 python -u bench.py --kernel-events timed --no-cpu-baseline --no-pods --no-parse --no-keyed > gpurun_out/bench_${TAG}_timed.json 2> gpurun_out/bench_${TAG}_timed.err || exit $?
bash scripts/gpu_emulate.sh $TAG C4 8 || exit $?
OUT=gpurun_out/prof_$TAG; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --no-cpu-baseline --no-dense --no-pods --no-parse --no-keyed --steps 20 > $OUT/trace.log 2>&1 || exit $?
python3 - <<PY
import json, csv, glob
for f in ['gpurun_out/bench_$TAG.json', 'gpurun_out/bench_${TAG}_timed.json', 'gpurun_out/emu_${TAG}_C4_w8.json']:
    d = json.load(open(f)); r = d['roofline_reduce']; v = d['roofline_valu']
    print(f.split('/')[-1], 'step %.4f' % d['ms_per_step'], 'red %.4f %.3f' % (r['ms_per_launch'], r['frac']), 'cold %.4f %.3f' % (r['ms_per_launch_cold'], r['frac_cold']), 'fit %.4f %.3f' % (v.get('ms_per_launch', d['roofline_fit']['ms_per_launch']), v['frac']))
for row in csv.DictReader(open(glob.glob('$OUT/trace/*kernel_stats.csv')[0])):
    if 'reduce_kernel<2' in row['Name'] or 'fit_kernel' in row['Name']:
        print('rocprof', row['Name'][:40], row['Calls'], '%.2f us' % (float(row['AverageNs']) / 1e3))
PY
