set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "reference or random_vs_oracle or golden" > gpurun_out/r05_u_pytest.log 2>&1 &&
timeout -k 10 300 python -u scripts/ab_debug.py --schedule reference --reps 3 default > gpurun_out/r05_u_ab_new.log 2>&1 &&
SA_LIB_PATH=$PWD/ab/SA_INIT_HIST=0/libsa_hip.so timeout -k 10 300 python -u scripts/ab_debug.py --schedule reference --reps 3 default > gpurun_out/r05_u_ab_old.log 2>&1 &&
timeout -k 10 300 python -u scripts/ab_debug.py --schedule reference --reps 3 default > gpurun_out/r05_u_ab_new2.log 2>&1
