#!/bin/bash
# Guarded GPU session: parity tests, then the bench at several pipeline depths.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 540 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for k in "$@"; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --chunks $k > gpurun_out/bench_k$k.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "bench k=$k rc=$rc"; tail -5 gpurun_out/bench_k$k.log; exit $rc; }
  python - "$k" <<'PY'
import json, sys
k = sys.argv[1]
line = [l for l in open(f"gpurun_out/bench_k{k}.log") if l.startswith("{")][-1]
d = json.loads(line)
print(f"chunks={k} value={d['value']:.4g} ms/step={d['ms_per_step']:.4f} fit_ms/launch={d['roofline']['ms_per_launch']:.4f} "
      f"red_ms/launch={d['roofline_reduce']['ms_per_launch']:.4f} pipeline={d['pipeline']}")
PY
done
