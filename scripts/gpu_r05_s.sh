set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/r05_s_pytest_gpu.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_s_smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r05_s_bench.log 2>&1 && timeout -k 10 300 python -u bench.py --kind degenerate --steps 2 --warmup 1 > gpurun_out/r05_s_bench_degenerate.log 2>&1
