set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 240 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "xq_second_pass" > gpurun_out/r05_c_pytest.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-reference-schedule > gpurun_out/r05_c_bench.log 2>&1
