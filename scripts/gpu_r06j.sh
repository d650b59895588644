#!/bin/bash
# Round 6 check of the tree: the GPU suite, smoke(), the default bench line (cold leg), the
# emulated 8-way C4 rank, then the rocprofv3 kernel trace and PMC passes of the default
# bench (the pmc_traffic.json the line's traffic fields read) incl. the read-request sizes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06j}
bash scripts/gpu_final.sh $TAG || exit $?
bash scripts/gpu_emulate.sh $TAG C4 8 || exit $?
OUT=gpurun_out/prof_$TAG; mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline --no-dense --no-cold"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B --steps 20 > $OUT/trace.log 2>&1 || exit $?
echo "trace ok"
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_SMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $pmc --output-format csv -d $OUT/pmc$i -o run -- $B --steps 5 --warmup 1 > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i ($pmc) failed rc=$?"; exit 3; }
  echo "pmc $i ok: $pmc"
done
python3 scripts/summarize_prof.py $OUT $OUT/summary.md > /dev/null && head -12 $OUT/summary.md
