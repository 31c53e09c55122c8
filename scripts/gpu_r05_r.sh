set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 200 hpc_suffix_array_amd/csrc/build/microbench_bucket 30 5 > gpurun_out/r05_r_mb_bucket.log 2>&1
