set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 360 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "multi_rank or eight_and_four or config4_shape or single_rank" > gpurun_out/r05_g_pytest.log 2>&1 && \
timeout -k 10 300 python -u scripts/sim_ranks.py --full --n 1073741824 --kind dna --worlds 2,4,8 --reps 2 --json-out gpurun_out/r05_g_sim_full.json > gpurun_out/r05_g_sim_full.log 2>&1 && \
timeout -k 10 200 python -u scripts/sim_ranks.py --n 4294967296 --kind byte256 --worlds 8 --reps 3 > gpurun_out/r05_g_sim_cfg4.log 2>&1
