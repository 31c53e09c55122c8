#!/bin/bash
# GPU box (bash scripts/ab_env.sh VAR=VALUE ...): the default headline bench
# (1 GiB DNA, packed schedule) with the default environment and with each
# VAR=VALUE, interleaved twice.
set -e
mkdir -p gpurun_out/abenv
for v in default "$@" default "$@"; do
  envs=()
  [ "$v" != default ] && envs=("$v")
  log=gpurun_out/abenv/$(echo "$v" | tr ':=/' '___').log
  env "${envs[@]}" timeout -k 10 120 python -u bench.py --no-cpu-baseline --no-reference-schedule --steps 10 --warmup 2 > "$log" 2>&1
  python - "$v" "$log" <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[2]) if l.startswith('{')][0])
k=d['kernels_ms_per_step']
print(sys.argv[1], d['ms_per_step'], d['verified'], ' '.join(f'{a}={b}' for a, b in k.items() if b))
PY
done
