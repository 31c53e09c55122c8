set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 bash scripts/ab_run.sh SA_TEXT_BLOCK=1024 > gpurun_out/r05_j_ab_text_block.log 2>&1
