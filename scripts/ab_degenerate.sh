set -e
mkdir -p gpurun_out/dab
for v in default SA_MAX_CHUNKS=16384 SA_MAX_CHUNKS=65536; do
  if [ "$v" = default ]; then unset SA_LIB_PATH; else export SA_LIB_PATH=$PWD/ab/$v/libsa_hip.so; fi
  timeout -k 10 120 python -u bench.py --no-cpu-baseline --kind degenerate --steps 1 --warmup 1 > gpurun_out/dab/$v.log 2>&1
  python -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/dab/$v.log') if l.startswith('{')][0])
k=d['kernels_ms_per_step']
print('$v', d['ms_per_step'], d['verified'], {x: k[x] for x in ('seg_count','seg_write','sort_u','scatter_keys')})
"
done
