#!/bin/bash
# GPU box (gpurun): bash scripts/gpu_steps.sh <tag> <step>...
# Each step runs under its own time limit and writes gpurun_out/<tag>_<step>.log;
# the first failing step ends the call (no later GPU step after a fault,
# abort or time limit).  Steps:
#   pytest       the full -m gpu suite (slow tests included)
#   pytest_fast  -m "gpu and not slow"
#   k:<expr>     -m gpu -k <expr>
#   smoke        __graft_entry__.smoke()
#   bench        bench.py (1 GiB DNA, CPU baseline, reference schedule)
#   bench_quick  bench.py without the CPU baseline and the reference schedule
#   dist1        bench.py --mode distributed (the range-partitioned driver at N = 1)
#   degenerate   bench.py --kind degenerate
#   kinds        bench.py for alnum / ascii127 / byte256

#   collect      rocprof summaries: DNA, degenerate, reference schedule
#   collect_dna  rocprof summary of the headline only
#   mb_bucket    microbench_bucket (the local sort alone, 2^30 items)
#   abcheck      scripts/ab_check.py 0 1 2 (checker level-1 bins 256 / 1024 / 512, and the LCP)
#   abk:<kind>:<v1,v2>  the same A/B on another alphabet
#   ab:<v1,v2>   scripts/ab_debug.py default v1 v2 (in-process interleaved A/B)
set -o pipefail
tag=${1:?tag}; shift
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out
run() {   # run <limit s> <log> <cmd...>
    local lim=$1 log=gpurun_out/${tag}_$2; shift 2
    echo "== $(date +%T) $log: $*"
    timeout -k 10 "$lim" "$@" > "$log" 2>&1
    local rc=$?
    tail -n 3 "$log"
    if [ $rc -ne 0 ]; then echo "step $log failed rc=$rc"; exit $rc; fi
}
for s in "$@"; do
    case $s in
    pytest) run 900 pytest_gpu.log python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu tests ;;
    pytest_fast) run 600 pytest_gpu_fast.log python -u -m pytest -v --timeout 200 --timeout-method thread -m "gpu and not slow" tests ;;
    k:*) e=${s#k:}; run 600 pytest_k.log python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu -k "$e" tests ;;
    smoke) run 120 smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run 300 bench_dna1g.log python -u bench.py ;;
    bench_quick) run 200 bench_quick.log python -u bench.py --no-cpu-baseline --no-reference-schedule ;;
    dist1) run 300 bench_dist1.log python -u bench.py --mode distributed --no-cpu-baseline ;;
    degenerate) run 300 bench_degenerate1g.log python -u bench.py --kind degenerate --no-cpu-baseline --no-reference-schedule ;;
    kinds) for k in alnum ascii127 byte256; do
               run 200 bench_$k.log python -u bench.py --kind $k --no-cpu-baseline --no-reference-schedule
           done ;;

    collect) run 900 collect_dna.log bash profiles/collect.sh ${tag} &&
             run 900 collect_deg.log bash profiles/collect.sh ${tag}_degenerate1g --kind degenerate &&
             run 900 collect_ref.log bash profiles/collect.sh ${tag}_refsched --schedule reference ;;
    collect_dna) run 900 collect_dna.log bash profiles/collect.sh ${tag} ;;
    mb_bucket) run 120 mb_bucket.log hpc_suffix_array_amd/csrc/build/microbench_bucket 30 5 ;;
    alnumk) for kk in 8 7; do
                run 200 bench_alnum_k$kk.log python -u bench.py --kind alnum --init-chars $kk --no-cpu-baseline --no-reference-schedule --no-lcp
            done ;;
    abcheck) run 300 ab_check.txt python -u scripts/ab_check.py 0 3 ;;
    abref:*) v=${s#abref:}; run 600 abref_${v//[,+]/_}.txt python -u scripts/ab_debug.py --schedule reference --reps 3 default ${v//,/ } ;;
    abk:*) v=${s#abk:}; kk=${v%%:*}; v=${v#*:}; run 300 ab_${kk}_${v//[,+]/_}.txt python -u scripts/ab_debug.py --kind $kk --reps 6 default ${v//,/ } ;;
    ab:*) v=${s#ab:}; run 300 ab_${v//[,+]/_}.txt python -u scripts/ab_debug.py --reps 6 default ${v//,/ } ;;
    *) echo "unknown step $s"; exit 2 ;;
    esac
done
