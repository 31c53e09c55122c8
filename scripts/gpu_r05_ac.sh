set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread -k "alphabet or golden or random_vs_oracle or distributed_hip_single or byte256" > gpurun_out/r05_ac_pytest.log 2>&1 &&
for k in dna alnum; do timeout -k 10 200 python -u scripts/ab_debug.py --kind $k --reps 4 default > gpurun_out/r05_ac_ab_$k.log 2>&1 || exit 1; done
