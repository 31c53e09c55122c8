set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash profiles/collect.sh r05_fin5 > gpurun_out/r05_fin5_collect_dna.log 2>&1 &&
bash profiles/collect.sh r05_fin5_degenerate1g --kind degenerate > gpurun_out/r05_fin5_collect_deg.log 2>&1 &&
bash profiles/collect.sh r05_fin5_refsched --schedule reference > gpurun_out/r05_fin5_collect_ref.log 2>&1
