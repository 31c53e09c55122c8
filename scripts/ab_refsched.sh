#!/bin/bash
# GPU box (bash scripts/ab_refsched.sh <variants>): the reference schedule
# (bench.py --schedule reference) for the working tree and each ab/<variant>,
# interleaved twice: ms per build and per doubling round.
set -e
mkdir -p gpurun_out/abref
for v in default "$@" default "$@"; do
  if [ "$v" = default ]; then unset SA_LIB_PATH; else export SA_LIB_PATH=$PWD/ab/$v/libsa_hip.so; fi
  timeout -k 10 150 python -u bench.py --schedule reference --no-cpu-baseline --no-reference-schedule --steps 3 --warmup 1 > gpurun_out/abref/$v.log 2>&1
  python - "$v" gpurun_out/abref/$v.log <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[2]) if l.startswith('{')][0])
print(sys.argv[1], d['ms_per_step'], d['verified'], 'rounds', d.get('ms_per_round'))
PY
done
