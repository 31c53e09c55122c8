#!/bin/bash
# GPU box (bash scripts/ab_sim.sh <variant>...): per-rank round 1 of the
# range-partitioned build (scripts/sim_ranks.py; default G = 8 on 1 GiB DNA,
# SIM_ARGS overrides the sim_ranks arguments) for the working tree ("new")
# and each ab/<variant>/libsa_hip.so, interleaved twice.
set -e
mkdir -p gpurun_out/absim
args=${SIM_ARGS:---worlds 8 --reps 5}
for v in new "$@" new "$@"; do
  if [ "$v" = new ]; then unset SA_LIB_PATH; else export SA_LIB_PATH=$PWD/ab/$v/libsa_hip.so; fi
  timeout -k 10 150 python -u scripts/sim_ranks.py $args > gpurun_out/absim/$v.log 2>&1
  echo $v $(grep -o "round1_ms\": [0-9.]*" gpurun_out/absim/$v.log | tr '\n' ' ')
done
