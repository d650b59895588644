set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for v in ${VARS:-rel dnr dns dnst dall}; do
  OUT=gpurun_out/prof_${TAG:-r06aa}_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
    python3 -u scripts/ab_variants.py run --keyed --config C4 --rounds 3 --reps 10 $v > $OUT.log 2>&1 || exit $?
  python3 -c "
import csv, glob
for row in csv.DictReader(open(glob.glob('$OUT/*kernel_stats.csv')[0])):
    if 'kb_' in row['Name']: print('$v', row['Calls'], '%.2f us' % (float(row['AverageNs']) / 1e3), row['Name'][:50])"
done
