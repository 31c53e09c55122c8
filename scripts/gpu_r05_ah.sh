set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/r05_ah_pytest_gpu.log 2>&1 &&
for i in 1 2; do
timeout -k 10 200 python -u scripts/ab_debug.py --reps 6 default no_key1_round > gpurun_out/r05_ah_ab_$i.log 2>&1 || exit 1
done
