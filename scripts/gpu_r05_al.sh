set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "key1 or sparse or bucketed or window or config or xq or pad" > gpurun_out/r05_al_pytest.log 2>&1 &&
bash scripts/ab_run.sh head > gpurun_out/r05_al_ab_1.log 2>&1 &&
bash scripts/ab_run.sh head > gpurun_out/r05_al_ab_2.log 2>&1
