#!/bin/bash
# GPU box: per-rank round-1 kernel times (scripts/sim_ranks.py under rocprofv3)
# for the default library and each ab/<variant>: bash scripts/ab_sim.sh <worlds> <variants...>
set -e
w=$1; shift
mkdir -p gpurun_out/abs
export TMPDIR=/tmp
for v in default "$@"; do
  if [ "$v" = default ]; then unset SA_LIB_PATH; else export SA_LIB_PATH=$PWD/ab/$v/libsa_hip.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abs/$v -o t -- python3 scripts/sim_ranks.py --worlds $w --reps 3 > gpurun_out/abs/$v.log 2>&1 || true
  python3 - "$v" <<'PY'
import csv, sys
v = sys.argv[1]
rows = list(csv.DictReader(open(f"gpurun_out/abs/{v}/t_kernel_stats.csv")))
print(v, " ".join(f"{r['Name'].split('(')[0].replace('void sa::', '')[:28]}={float(r['AverageNs'])/1e6:.3f}" for r in rows
                 if any(k in r['Name'] for k in ('bucket_hist', 'split_list', 'split_seg', 'bucket_sort<', 'split_text'))))
PY
  grep world gpurun_out/abs/$v.log | tail -1
done
