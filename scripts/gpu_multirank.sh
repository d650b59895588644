#!/bin/bash
# Rehearse the multi-rank bench path on a 1-GPU box: N=1 reference, then 2 ranks sharing
# the GPU over gloo (RCCL refuses two ranks on one device; the default p2p exchange maps
# the ranks' mailboxes through IPC handles).  The totals checksum must match.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
CFG=${1:-C3}
timeout -k 10 300 python -u bench.py --config $CFG --no-cpu-baseline --steps 5 --scaling strong > gpurun_out/mr_n1.log 2>&1 || exit $?
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --config $CFG \
  --dist-backend gloo --steps 5 --scaling strong > gpurun_out/mr_n2.log 2>&1 || exit $?
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --config $CFG \
  --dist-backend gloo --steps 5 --scaling weak > gpurun_out/mr_n2w.log 2>&1 || exit $?
python - <<'PY'
import json
a = json.loads(open("gpurun_out/mr_n1.log").read().strip().splitlines()[-1])
b = json.loads(open("gpurun_out/mr_n2.log").read().strip().splitlines()[-1])
print("n1", a["value"], a["totals_checksum"], a["n_gpus"])
print("n2", b["value"], b["totals_checksum"], b["n_gpus"], b["config"]["parallelism"],
      b["world"]["exchange"], b["world"]["exchange_note"], b.get("exchange_check"),
      "exchange ms", b["allreduce_ms"])
assert a["totals_checksum"] == b["totals_checksum"], "sharded totals differ"
assert b.get("exchange_check", {}).get("equals_allreduce_finalize", True), "p2p exchange differs"
w = json.loads(open("gpurun_out/mr_n2w.log").read().strip().splitlines()[-1])
print("n2 weak", w["value"], w["scaling"], w["config"]["nodes"])
assert w["scaling"] == "weak" and w["config"]["nodes"] == 2 * a["config"]["nodes"]
print("MULTIRANK OK")
PY
