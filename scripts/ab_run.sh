#!/bin/bash
# GPU box (bash scripts/ab_run.sh <variants>): bench the default library and each ab/<variant>, interleaved
set -e
mkdir -p gpurun_out/ab
for v in default "$@" default "$@"; do
  if [ "$v" = default ]; then unset SA_LIB_PATH; else export SA_LIB_PATH=$PWD/${AB_DIR:-ab}/$v/libsa_hip.so; fi
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-reference-schedule --steps 10 --warmup 2 > gpurun_out/ab/$v.log 2>&1
  python - "$v" gpurun_out/ab/$v.log <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[2]) if l.startswith('{')][0])
k=d['kernels_ms_per_step']
print(sys.argv[1], d['ms_per_step'], d['verified'], 'alpha', k['alphabet'], 'hist', k['pack'], 'first', k['scatter_first'], 'second', k['scatter_keys'], 'local', k['local_sort'], 'u', k['sort_u'])
PY
done
