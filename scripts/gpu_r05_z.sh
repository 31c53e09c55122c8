set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/r05_z_pytest_gpu.log 2>&1 &&
for i in 1 2; do
timeout -k 10 200 python -u scripts/ab_debug.py --reps 8 default > gpurun_out/r05_z_ab_new$i.log 2>&1 &&
SA_LIB_PATH=$PWD/ab/prev/libsa_hip.so timeout -k 10 200 python -u scripts/ab_debug.py --reps 8 default > gpurun_out/r05_z_ab_prev$i.log 2>&1 || exit 1
done
