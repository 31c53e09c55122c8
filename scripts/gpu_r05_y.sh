set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
d=gpurun_out/r05_y
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $d -o tr -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-reference-schedule > gpurun_out/r05_y.log 2>&1
cp $(find $d -name "*kernel_trace.csv" | head -1) gpurun_out/r05_y_trace.csv
