#!/bin/bash
# GPU box: 1 GiB builds of every alphabet, default library vs ab/<variant>
for k in alnum ascii127 byte256 dna; do
  for v in default "$@"; do
    if [ "$v" = default ]; then unset SA_LIB_PATH; else export SA_LIB_PATH=$PWD/ab/$v/libsa_hip.so; fi
    timeout -k 10 120 python -u bench.py --kind $k --no-cpu-baseline --no-reference-schedule --steps 5 --warmup 1 > gpurun_out/abk_$k_$v.log 2>&1
    python3 - "$k" "$v" gpurun_out/abk_$k_$v.log <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[3]) if l.startswith('{')][0])
k=d['kernels_ms_per_step']
print(sys.argv[1], sys.argv[2], d['ms_per_step'], d['verified'], 'alpha', k['alphabet'], 'first', k['scatter_first'], 'second', k['scatter_keys'], 'local', k['local_sort'], 'u', k['sort_u'], 'rounds', d['rounds'])
PY
  done
done
