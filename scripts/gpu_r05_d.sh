set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/ab_debug.py --reps 6 default no_xq > gpurun_out/r05_d_ab_xq.log 2>&1
