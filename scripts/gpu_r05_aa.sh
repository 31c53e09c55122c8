set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "byte256 or round1 or golden or random_vs_oracle" > gpurun_out/r05_aa_pytest.log 2>&1 &&
for i in 1 2; do
timeout -k 10 200 python -u scripts/ab_debug.py --kind byte256 --reps 6 default > gpurun_out/r05_aa_ab_new$i.log 2>&1 &&
SA_LIB_PATH=$PWD/ab/SA_TEXT_IDENT=0/libsa_hip.so timeout -k 10 200 python -u scripts/ab_debug.py --kind byte256 --reps 6 default > gpurun_out/r05_aa_ab_old$i.log 2>&1 || exit 1
done
