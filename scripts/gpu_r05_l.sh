set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
SA_LIB_PATH=$PWD/ab/SA_LSD_PROF=1/libsa_hip.so timeout -k 10 300 python -u scripts/ab_debug.py --schedule reference --reps 1 default > gpurun_out/r05_l_lsd_prof.log 2>&1
