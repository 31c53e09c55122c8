set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
d=gpurun_out/r05_t
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o sim -- python3 scripts/sim_ranks.py --n 1073741824 --kind dna --worlds 8 --reps 2 > gpurun_out/r05_t_sim8.log 2>&1
cp $(find $d -name "*kernel_stats.csv" | head -1) gpurun_out/r05_t_sim8_kernel_stats.csv
