#!/bin/bash
# GPU box: local-sort variants on the config-2 text (64 MiB DNA) with SA_TRACE
for v in default "$@"; do
  if [ "$v" = default ]; then unset SA_LIB_PATH; else export SA_LIB_PATH=$PWD/ab/$v/libsa_hip.so; fi
  echo "== $v"
  SA_TRACE=1 timeout -k 10 120 python -u bench.py --n 67108864 --no-cpu-baseline --no-reference-schedule --steps 1 --warmup 0 2>&1 | grep -E "bucketed round 1:|verified" | sed 's/.*"verified": \([a-z]*\).*/verified \1/' | tail -3
done
