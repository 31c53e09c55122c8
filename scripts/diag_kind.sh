#!/bin/bash
# GPU box: SA_TRACE of one 1 GiB build of --kind $1 for the default library and each ab/<variant>
k=$1; shift
for v in default "$@"; do
  if [ "$v" = default ]; then unset SA_LIB_PATH; else export SA_LIB_PATH=$PWD/ab/$v/libsa_hip.so; fi
  echo "== $v"
  SA_TRACE=1 timeout -k 10 120 python -u bench.py --kind $k --no-cpu-baseline --no-reference-schedule --steps 1 --warmup 0 2>&1 | grep -E "bucketed round 1:|round h=|local_sort" | sed 's/"kernels_gbs.*//' | head -5
done
