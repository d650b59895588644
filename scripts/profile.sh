#!/bin/bash
# rocprofv3 kernel trace + separate PMC passes of the default bench workload.
# Usage (on the GPU box): bash scripts/profile.sh <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline --no-dense"
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run \
  -- $B --steps 20 > $OUT/trace.log 2>&1 || exit $?
echo "trace ok"
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_CVT SQ_INSTS_LDS SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $pmc --output-format csv -d $OUT/pmc$i -o run \
    -- $B --steps 5 --warmup 1 > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i ($pmc) failed rc=$?"; exit 3; }
  echo "pmc $i ok: $pmc"
done
