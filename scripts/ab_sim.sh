#!/bin/bash
# GPU box (bash scripts/ab_sim.sh <variant>...): per-rank round 1 of the
# range-partitioned build at G = 8 (scripts/sim_ranks.py, 1 GiB DNA) for the
# working tree ("new") and each ab/<variant>/libsa_hip.so, interleaved twice.
set -e
mkdir -p gpurun_out/absim
for v in new "$@" new "$@"; do
  if [ "$v" = new ]; then unset SA_LIB_PATH; else export SA_LIB_PATH=$PWD/ab/$v/libsa_hip.so; fi
  timeout -k 10 100 python -u scripts/sim_ranks.py --worlds 8 --reps 5 > gpurun_out/absim/$v.log 2>&1
  echo $v $(grep -o "round1_ms\": [0-9.]*" gpurun_out/absim/$v.log | tr '\n' ' ')
done
