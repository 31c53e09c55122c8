set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "pivot or degenerate or periodic or round1_fallback" > gpurun_out/r05_m_pytest.log 2>&1 &&
timeout -k 10 300 python -u scripts/ab_debug.py --kind degenerate --reps 2 default no_tied > gpurun_out/r05_m_ab_tied.log 2>&1
