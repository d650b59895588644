#!/bin/bash
# Round 4: does the GPU's clock ramp reach into the timed steps?  The default bench line
# (side legs now warmed for >= 0.1 s each) and the step after a 300 ms dummy load, twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04r}
mkdir -p gpurun_out
timeout -k 10 240 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
python3 -c "
import json;d=json.load(open('gpurun_out/bench_$TAG.json'))
print('default step', d['ms_per_step'], 'reduce', d['roofline_reduce']['ms_per_launch'], 'keyed', d['keyed']['ms_per_launch'], d['keyed']['roofline']['frac'], 'pods', d['pods']['ms_per_launch'], 'cpu', d['parse']['ms_per_launch'], 'qty', d['parse']['quantity']['ms_per_launch'], d['parse']['quantity']['roofline']['frac'])"
F="--no-cpu-baseline --no-keyed --no-pods --no-parse --no-dense"
for rep in 1 2; do
  for pw in 0 300; do
    timeout -k 10 200 python -u bench.py $F --prewarm-ms $pw > gpurun_out/b_${TAG}_pw${pw}_$rep.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/b_${TAG}_pw${pw}_$rep.json'));print('prewarm $pw', d['ms_per_step'], d['roofline_reduce']['ms_per_launch'])"
  done
done
