set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "alphabet or kind or sigma or key1 or bucketed" > gpurun_out/r05_am_pytest.log 2>&1 &&
bash scripts/ab_kinds.sh head > gpurun_out/r05_am_kinds.log 2>&1 &&
bash scripts/ab_run.sh head > gpurun_out/r05_am_ab_1.log 2>&1
