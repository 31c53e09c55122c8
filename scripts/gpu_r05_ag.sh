set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 200 python -u scripts/ab_debug.py --reps 4 default > gpurun_out/r05_ag_2048_$i.log 2>&1 &&
SA_LIB_PATH=$PWD/ab/SA_ALPHA_GRID=4096/libsa_hip.so timeout -k 10 200 python -u scripts/ab_debug.py --reps 4 default > gpurun_out/r05_ag_4096_$i.log 2>&1 &&
SA_LIB_PATH=$PWD/ab/SA_ALPHA_GRID=8192/libsa_hip.so timeout -k 10 200 python -u scripts/ab_debug.py --reps 4 default > gpurun_out/r05_ag_8192_$i.log 2>&1 || exit 1
done
