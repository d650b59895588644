#!/bin/bash
# Round-end check of the committed tree, as the driver runs it: the whole -m gpu suite,
# smoke(), the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-final}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
timeout -k 10 240 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
python3 -c "
import json;d=json.load(open('gpurun_out/bench_$TAG.json'))
print('step', d['ms_per_step'], 'value %.4g'%d['value'], 'roofline', d['roofline']['frac'], 'traffic', d['roofline']['traffic'], 'keyed', d['keyed']['roofline']['frac'], 'qty', d['parse']['quantity']['roofline']['frac'], 'cpu', d['cpu_baseline']['value'], d['cpu_baseline']['match'], 'chk', d['totals_checksum'])"
