set -e
mkdir -p gpurun_out/ab
for v in default head default head; do
  if [ "$v" = default ]; then unset SA_LIB_PATH; else export SA_LIB_PATH=$PWD/abx/$v/libsa_hip.so; fi
  for k in alnum ascii127; do
    timeout -k 10 120 python -u bench.py --kind $k --no-cpu-baseline --no-reference-schedule --no-lcp --steps 10 --warmup 2 > gpurun_out/ab/${v}_$k.log 2>&1
    python - "$v $k" gpurun_out/ab/${v}_$k.log <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[2]) if l.startswith('{')][0])
k=d['kernels_ms_per_step']
print(sys.argv[1], d['ms_per_step'], d['verified'], 'first', k['scatter_first'], 'second', k['scatter_keys'], 'local', k['local_sort'])
PY
  done
done
