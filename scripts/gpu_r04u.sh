#!/bin/bash
# Round 4: size-dependent placement of the spec ranks' workgroups (behind the reduce's at
# >= 16M containers): the reduce parity tests, bench lines at C4 and rank 0 of an 8-way split.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r04u}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shards_configs.py -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
F="--no-cpu-baseline --no-keyed --no-pods --no-parse --no-dense"
for rep in 1 2; do
  timeout -k 10 200 python -u bench.py $F > gpurun_out/b_${TAG}_$rep.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/b_${TAG}_$rep.json'));print('C4', round(d['ms_per_step'],5), 'reduce', round(d['roofline_reduce']['ms_per_launch'],5), round(d['roofline_reduce']['frac'],4), d['totals_checksum'])"
  timeout -k 10 200 python -u bench.py $F --emulate-world 8 --steps 50 > gpurun_out/b_${TAG}_w8_$rep.json 2>/dev/null || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/b_${TAG}_w8_$rep.json'));print('C4/8', round(d['ms_per_step'],5), 'reduce', round(d['roofline_reduce']['ms_per_launch'],5), d['totals_checksum'])"
done
