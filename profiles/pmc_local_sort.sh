#!/bin/bash
# SQ counters of the bucketed first round's kernels (run on the GPU box):
#   bash profiles/pmc_local_sort.sh <tag> [bench args...]
set -uo pipefail
tag=${1:?tag}; shift
out=gpurun_out/pmc_$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
    --output-format csv -d "$out/sq" -o sq -- python3 bench.py --no-cpu-baseline --no-profile --steps 1 --warmup 0 "$@" > "$out/sq.log" 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH \
    --output-format csv -d "$out/sq2" -o sq2 -- python3 bench.py --no-cpu-baseline --no-profile --steps 1 --warmup 0 "$@" > "$out/sq2.log" 2>&1 || exit $?
python3 - "$out" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(out + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0][:60]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in acc.items():
    if any(s in k for s in ("bucket_sort", "onesweep", "k_split", "bucket_hist", "seg_")):
        print(k)
        for c, x in sorted(v.items()):
            print(f"   {c:24s} {x:.4g}")
PY
