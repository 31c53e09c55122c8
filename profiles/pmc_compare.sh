#!/bin/bash
# SQ counters of k_bucket_sort in the real build (bench.py) and in the
# synthetic microbenchmark (uniform keys), same counter sets:
#   bash profiles/pmc_compare.sh <tag>
set -uo pipefail
tag=${1:?tag}
out=gpurun_out/pmcc_$tag
mkdir -p "$out"
export TMPDIR=/tmp
S1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES"
S2="SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_ANY"
for set in 1 2; do
  eval "C=\$S$set"
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$out/b$set" -o b -- python3 bench.py --no-cpu-baseline --no-profile --steps 1 --warmup 0 > "$out/b$set.log" 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d "$out/m$set" -o m -- hpc_suffix_array_amd/csrc/build/microbench_bucket 30 1 28 > "$out/m$set.log" 2>&1 || exit $?
done
python3 - "$out" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for src in ("b", "m"):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{out}/{src}[12]/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            if "k_bucket_sort<1024, 18, 0>" in k:
                acc[r["Dispatch_Id"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("bench" if src == "b" else "microbench (uniform 28-bit keys)")
    for d, v in list(acc.items())[:2]:
        print("  dispatch", d, {c: f"{sum(x):.4g}" for c, x in sorted(v.items())})
PY
