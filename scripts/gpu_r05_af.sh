set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "pivot or degenerate or periodic or round1_fallback or alphabet_late or random_vs_oracle" > gpurun_out/r05_af_pytest.log 2>&1 &&
timeout -k 10 300 python -u scripts/ab_debug.py --kind degenerate --reps 2 default > gpurun_out/r05_af_ab_new.log 2>&1 &&
SA_LIB_PATH=$PWD/ab/SA_PIVOT_MERGED=0/libsa_hip.so timeout -k 10 300 python -u scripts/ab_debug.py --kind degenerate --reps 2 default > gpurun_out/r05_af_ab_old.log 2>&1
