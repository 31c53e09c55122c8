set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
d=gpurun_out/r05_n
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 scripts/ab_debug.py --kind degenerate --reps 1 default > gpurun_out/r05_n.log 2>&1
f=$(find $d -name "*kernel_stats.csv" | head -1)
cp $f gpurun_out/r05_n_kernel_stats.csv
