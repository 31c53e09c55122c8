set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 500 hpc_suffix_array_amd/csrc/build/microbench_place > gpurun_out/r05_x_mb_place.log 2>&1
