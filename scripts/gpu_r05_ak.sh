set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash scripts/ab_run.sh SA_LAZY_SAMPLES=1 SA_LAZY_SAMPLES=0 head > gpurun_out/r05_ak_ab_1.log 2>&1 &&
bash scripts/ab_run.sh SA_LAZY_SAMPLES=1 SA_LAZY_SAMPLES=0 head > gpurun_out/r05_ak_ab_2.log 2>&1
