#!/bin/bash
# A/B of a variants/ build against the in-tree library through the bench's emulated ranks
# (the capacity entry points the A/B harness does not drive): base, variant, base again.
#   bash scripts/gpu_ab_lib.sh <tag> <variant> <W>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; VAR=$2; shift 2
mkdir -p gpurun_out
cp kubernetesclustercapacity_amd/libkcc.so /tmp/libkcc_base.so
run() {  # $1: label
  for W in "$@"; do :; done
}
for round in base $VAR base2 ${VAR}2; do
  case $round in base|base2) cp /tmp/libkcc_base.so kubernetesclustercapacity_amd/libkcc.so ;;
                 *) cp variants/libkcc_$VAR.so kubernetesclustercapacity_amd/libkcc.so ;; esac
  for W in "$@"; do
    OUT=gpurun_out/abl_${TAG}_${round}_w$W.json
    timeout -k 10 200 python3 -u bench.py --config C4 --scaling strong --emulate-world $W \
      --no-cpu-baseline --no-keyed --no-pods --no-parse --no-dense --steps 100 --warmup 10 \
      > $OUT 2> ${OUT%.json}.err || exit $?
    echo "$round W=$W $(grep -o '"ms_per_step": [0-9.]*' $OUT) fit $(python3 -c "import json;print(round(json.load(open('$OUT'))['pipeline']['fit_ms_per_step']*1e3,2))")"
  done
done
cp /tmp/libkcc_base.so kubernetesclustercapacity_amd/libkcc.so
