set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r05_f_prof -o r05_f -- python3 $GRAFT_REPO_ROOT/scripts/ab_debug.py --reps 3 default > $GRAFT_REPO_ROOT/gpurun_out/r05_f.log 2>&1
