#!/bin/bash
# GPU box (bash scripts/ab_ref.sh <variants>): the reference schedule
# (bench.py --schedule reference) with the default library and each
# ab/<variant> (scripts/ab_build_variants.sh), interleaved.  A variant named
# env:NAME=VALUE runs the default library with that environment variable.
set -e
mkdir -p gpurun_out/abref
for v in default "$@" default "$@"; do
  unset SA_LIB_PATH
  envs=()
  case "$v" in
    default) ;;
    env:*) envs=("${v#env:}") ;;
    *) export SA_LIB_PATH=$PWD/ab/$v/libsa_hip.so ;;
  esac
  log=gpurun_out/abref/$(echo "$v" | tr ':=/' '___').log
  env "${envs[@]}" timeout -k 10 120 python -u bench.py --schedule reference --no-cpu-baseline --steps 3 --warmup 1 > "$log" 2>&1
  python - "$v" "$log" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[2]) if l.startswith('{')][0])
k=d['kernels_ms_per_step']
print(sys.argv[1], d['ms_per_step'], d['verified'], 'rounds', d['ms_per_round'], 'passes', d['passes_per_round'],
      {x: k[x] for x in ('hist_first', 'scatter_first', 'scatter_keys', 'heads', 'rerank') if k.get(x)})
PY
done
