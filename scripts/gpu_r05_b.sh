set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 240 ./hpc_suffix_array_amd/csrc/build/microbench_seg > gpurun_out/r05_b_mb_seg.log 2>&1 && \
for k in alnum ascii127 byte256; do
  timeout -k 10 120 python -u bench.py --kind $k --steps 10 --warmup 3 --no-reference-schedule --no-cpu-baseline > gpurun_out/r05_b_bench_$k.log 2>&1 || exit 1
done
