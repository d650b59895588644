#!/bin/bash
# Round 6: reduce A/B (forward prefixes) and keyed-gather A/B (gold = round 5's gather,
# ga0 = XCD-placed gather with last-part-only combine, gapipe = + pipelined sub-batches),
# the keyed GPU tests on the release library, then the keyed leg's PMC passes incl. the
# read-request size breakdown.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r06d}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_keyed.py tests/test_abi_inlib.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_variants.py run --keyed --config C4 --rounds 5 --reps 10 gold ga0 gapipe > gpurun_out/ab_${TAG}_keyed.txt 2>&1 || exit $?
grep -h '^{' gpurun_out/ab_${TAG}_keyed.txt
bash scripts/gpu_ab.sh ${TAG}red base fwd || exit $?
OUT=gpurun_out/prof_$TAG; mkdir -p $OUT
B="python3 bench.py --no-cpu-baseline --no-dense --no-pods --no-parse --no-cold"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B --steps 10 > $OUT/trace.log 2>&1 || exit $?
echo "trace ok"
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $pmc --output-format csv -d $OUT/pmc$i -o run -- $B --steps 3 --warmup 1 > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i ($pmc) failed rc=$?"; exit 3; }
  echo "pmc $i ok: $pmc"
done
python3 scripts/summarize_prof.py $OUT $OUT/summary.md > /dev/null && grep -E "kb_|reduce_kernel|RDREQ" $OUT/summary.md | head -20
