set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_ab.sh r04e base prio prio2 diag_redld || exit $?
timeout -k 10 200 python -u scripts/probe/timeline.py tl --config C4 > gpurun_out/tl_r04e_c4.txt 2>&1 || exit $?
timeout -k 10 200 python -u scripts/probe/timeline.py tlprio --config C4 > gpurun_out/tl_r04e_c4prio.txt 2>&1 || exit $?
grep "^reduce" gpurun_out/tl_r04e_c4.txt gpurun_out/tl_r04e_c4prio.txt
