set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "alphabet_late or pivot_round1 or degenerate" > gpurun_out/r05_ad_pytest.log 2>&1
