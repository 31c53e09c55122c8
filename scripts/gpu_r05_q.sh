set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "pivot or degenerate or periodic or round1_fallback" > gpurun_out/r05_q_pytest.log 2>&1 &&
timeout -k 10 300 python -u scripts/ab_debug.py --kind degenerate --reps 2 default no_tied > gpurun_out/r05_q_ab_tied.log 2>&1 &&
d=gpurun_out/r05_q &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 scripts/ab_debug.py --kind degenerate --reps 1 default > gpurun_out/r05_q.log 2>&1 &&
cp $(find $d -name "*kernel_stats.csv" | head -1) gpurun_out/r05_q_kernel_stats.csv
