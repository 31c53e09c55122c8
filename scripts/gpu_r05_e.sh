set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/ab_debug.py --reps 6 default no_xq > gpurun_out/r05_e_ab_xq.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "xq_second_pass" > gpurun_out/r05_e_pytest.log 2>&1
