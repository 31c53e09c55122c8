#!/bin/bash
# GPU box (bash scripts/ab_kstats.sh <pattern> <variant>...): rocprofv3 kernel
# stats of sim_ranks --worlds 8 for the working tree and each ab/<variant>,
# printing the average duration of the kernels whose name matches <pattern>.
set -e
pat=$1; shift
export TMPDIR=/tmp
for v in new "$@"; do
  if [ "$v" = new ]; then unset SA_LIB_PATH; else export SA_LIB_PATH=$PWD/ab/$v/libsa_hip.so; fi
  d=gpurun_out/abk/$(echo "$v" | tr '=' '_')
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 scripts/sim_ranks.py --worlds 8 --reps 2 > /dev/null 2>&1
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  python3 - "$v" "$f" "$pat" <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[2])):
    if sys.argv[3] in x['Name']:
        print(sys.argv[1], x['Name'][:60], x['Calls'], round(float(x['AverageNs']) / 1e3, 1), 'us')
PY
done
