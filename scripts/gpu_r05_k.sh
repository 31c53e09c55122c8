set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "reference_lsd_queues or random_vs_oracle or rerank_permutation or radix_algorithms or degenerate or config2 or periodic" > gpurun_out/r05_k_pytest.log 2>&1 && \
timeout -k 10 300 python -u scripts/ab_debug.py --schedule reference --reps 3 default no_xq > gpurun_out/r05_k_ab_ref.log 2>&1
