#!/bin/bash
# Round 5: keyed 6-byte records, second cut (8-B LDS stage packed in LDS; aligned dword
# gather loads): tests, A/B vs round 4's records, per-kernel times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r05n}
bash scripts/gpu_r05l.sh $TAG && bash scripts/gpu_r05m.sh $TAG
