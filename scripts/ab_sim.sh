set -e
mkdir -p gpurun_out/absim
for v in head new head new; do
  if [ $v = head ]; then export SA_LIB_PATH=$PWD/ab/head/libsa_hip.so; else unset SA_LIB_PATH; fi
  timeout -k 10 100 python -u scripts/sim_ranks.py --worlds 8 --reps 5 > gpurun_out/absim/$v.log 2>&1
  echo $v $(grep -o "round1_ms\": [0-9.]*" gpurun_out/absim/$v.log | tr '\n' ' ')
done
unset SA_LIB_PATH
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/absim/prof_new -o run -- python3 scripts/sim_ranks.py --worlds 8 --reps 3 > /dev/null 2>&1
SA_LIB_PATH=$PWD/ab/head/libsa_hip.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/absim/prof_head -o run -- python3 scripts/sim_ranks.py --worlds 8 --reps 3 > /dev/null 2>&1
for v in new head; do echo == $v; f=$(find gpurun_out/absim/prof_$v -name "*kernel_stats.csv" | head -1); python3 -c "import csv,sys; r=list(csv.DictReader(open(sys.argv[1]))); [print(x[\"Name\"][:60], x[\"Calls\"], x[\"AverageNs\"]) for x in r[:14]]" $f; done
