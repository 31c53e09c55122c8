set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
SA_LIB_PATH=$PWD/ab/SA_LS_HRANK=1/libsa_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "bucketed or round1 or random_vs_oracle or local_sort or golden" > gpurun_out/r05_ae_pytest.log 2>&1 &&
for i in 1 2; do
SA_LIB_PATH=$PWD/ab/SA_LS_HRANK=1/libsa_hip.so timeout -k 10 200 python -u scripts/ab_debug.py --reps 8 default > gpurun_out/r05_ae_ab_new$i.log 2>&1 &&
timeout -k 10 200 python -u scripts/ab_debug.py --reps 8 default > gpurun_out/r05_ae_ab_old$i.log 2>&1 || exit 1
done
