#!/bin/bash
# Run on the GPU box (via gpurun) from the repo root:
#   bash profiles/collect.sh <tag> [bench args...]
# 1. kernel trace + stats of the bench command (per-kernel average durations)
# 2. FETCH_SIZE pass, 3. WRITE_SIZE pass (separate --pmc passes: on gfx950
#    FETCH_SIZE takes 3 of the 4 TCC counter slots, WRITE_SIZE 2)
# then profiles/summarize.py writes profiles/<tag>_summary.json and copies the
# stats CSV into profiles/.
set -euo pipefail
tag=${1:?tag}; shift
args=("$@")
out=gpurun_out/prof_$tag
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o trace -- \
    python3 bench.py --no-cpu-baseline --no-reference-schedule --json-out "$out/bench.json" "${args[@]}" > "$out/trace.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o fetch -- \
    python3 bench.py --no-cpu-baseline --no-reference-schedule --no-profile "${args[@]}" --steps 1 --warmup 0 > "$out/fetch.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o write -- \
    python3 bench.py --no-cpu-baseline --no-reference-schedule --no-profile "${args[@]}" --steps 1 --warmup 0 > "$out/write.log" 2>&1
# 4. SQ pass: instruction mix, LDS bank conflicts and busy cycles (8 SQ counters, one pass)
if [ -z "${NO_SQ:-}" ]; then
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
    SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d "$out/sq" -o sq -- \
    python3 bench.py --no-cpu-baseline --no-reference-schedule --no-profile "${args[@]}" --steps 1 --warmup 0 > "$out/sq.log" 2>&1
fi
python3 profiles/summarize.py "$tag" "$out" "${args[@]}"
