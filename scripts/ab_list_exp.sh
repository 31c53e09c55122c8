set -e
mkdir -p gpurun_out/abl
export TMPDIR=/tmp
for v in default SA_LIST_EXP=1 SA_LIST_EXP=2 SA_LIST_EXP=3; do
  if [ "$v" = default ]; then unset SA_LIB_PATH; else export SA_LIB_PATH=$PWD/ab/$v/libsa_hip.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abl/$v -o t -- python3 scripts/sim_ranks.py --worlds 8 --reps 3 > gpurun_out/abl/$v.log 2>&1 || true
done
