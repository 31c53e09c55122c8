set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests > gpurun_out/r05_fin5_pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_fin5_smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r05_fin5_bench_dna1g.log 2>&1 &&
timeout -k 10 300 python -u bench.py --kind degenerate > gpurun_out/r05_fin5_bench_degenerate1g.log 2>&1 &&
for k in alnum ascii127 byte256; do timeout -k 10 200 python -u bench.py --kind $k --no-cpu-baseline --no-reference-schedule > gpurun_out/r05_fin5_bench_$k.log 2>&1 || exit 1; done
