#!/usr/bin/env python3
"""Multi-GPU scaling harness: the shape of the reference's MPI sweep
(scripts/benchmark_mpi.py:133-229 -- one run per process count, speedup and
efficiency columns, a summary table) and of its CUDA sweep
(benchmark_cuda_kaggle.py:200-289 -- speedup_vs_cpu), over MI355X GPUs.

Each configuration runs bench.py (one process per GPU; N > 1 through
torch.distributed.run on 127.0.0.1, RCCL) on the seeded synthetic text of
SURVEY.md 8(d) and reads its JSON line.  Columns follow mpi_results.csv
(file, size_bytes, size_mb, backend, processes, time_seconds, sa_time,
lcp_time, speedup, efficiency) plus suffixes_per_s and speedup_vs_cpu:
  * speedup    = sa_time at 1 GPU / sa_time at N GPUs (the reference divides
                 by the sequential CSV's sa_time; the 1-GPU run is this
                 harness's baseline, sequential_results.csv is used when it
                 has the same workload name),
  * efficiency = speedup / N,
  * speedup_vs_cpu = suffixes/s over the single-thread CPU baseline that
                 bench.py times on the 1-GPU run.
lcp_time is not measured here (bench.py times the SA build only) and is 0.

  python scripts/benchmark_scaling.py [--gpus 1,2,4,8] [--n 1073741824]
  python scripts/benchmark_scaling.py --dry-run    # print the commands only
"""
import argparse
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

COLUMNS = ["file", "size_bytes", "size_mb", "backend", "processes", "time_seconds", "sa_time", "lcp_time",
           "suffixes_per_s", "speedup", "efficiency", "speedup_vs_cpu"]


def command(n_gpus, args, port):
    bench = [os.path.join(ROOT, "bench.py"), "--gpus", str(n_gpus), "--steps", str(args.steps), "--warmup",
             str(args.warmup), "--n", str(args.n), "--kind", args.kind]
    if n_gpus > 1 or args.no_cpu_baseline:
        bench.append("--no-cpu-baseline")
    if n_gpus == 1:
        return [sys.executable] + bench
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n_gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port)] + bench


def last_json(text):
    for line in reversed(text.strip().splitlines()):
        line = line.strip()
        if line.startswith("{") and line.endswith("}"):
            return json.loads(line)
    raise ValueError("no JSON line in the bench output")


def rejected(r):
    """Why a bench.py line cannot enter the speedup / efficiency table (None
    when it can): an unverified suffix array, or a weak-scaling (replicas)
    run -- the reference's sweep divides ONE workload over the processes
    (benchmark_mpi.py:191-210)."""
    if r.get("verified") is not True:
        return f"suffix array not verified: {r.get('verified')}"
    if r.get("scaling") != "strong":
        return f"scaling {r.get('scaling')!r}: speedup / efficiency need one string over all GPUs"
    return None


def rows_from(results, workload, n, seq_sa_time=None):
    """results: [(N, bench JSON)] -> CSV rows with speedup/efficiency."""
    base = {N: r for N, r in results}
    t1 = seq_sa_time if seq_sa_time else (base[1]["ms_per_step"] / 1e3 if 1 in base else None)
    cpu = base[1].get("cpu_baseline", {}).get("value") if 1 in base else None
    rows = []
    for N, r in results:
        t = r["ms_per_step"] / 1e3
        speedup = t1 / t if t1 and t > 0 else 0.0
        rows.append({
            "file": workload, "size_bytes": n, "size_mb": n / (1 << 20), "backend": f"hip_{N}",
            "processes": N, "time_seconds": t, "sa_time": t, "lcp_time": 0.0,
            "suffixes_per_s": r["value"], "speedup": speedup, "efficiency": speedup / N if N else 0.0,
            "speedup_vs_cpu": r["value"] / cpu if cpu else 0.0,
        })
    return rows


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--gpus", default="1,2,4,8", help="comma-separated GPU counts")
    ap.add_argument("--n", type=int, default=1 << 30)
    ap.add_argument("--kind", default="dna")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--out", default=os.path.join(ROOT, "results", "csv", "gpu_scaling_results.csv"))
    ap.add_argument("--timeout", type=int, default=900, help="seconds per configuration")
    ap.add_argument("--dry-run", action="store_true")
    args = ap.parse_args(argv)
    counts = [int(x) for x in args.gpus.split(",") if x.strip()]
    if not args.dry_run:
        import torch
        have = torch.cuda.device_count()
        skipped = [N for N in counts if N > have]
        counts = [N for N in counts if N <= have]
        for N in skipped:
            print(f"  HIP-{N:2} GPU - NON DISPONIBILE ({have} visible)")
    workload = f"{args.kind}_{args.n}"
    print("BENCHMARK GPU SCALING - Suffix Array")
    print("=" * 60)
    results = []
    for i, N in enumerate(counts):
        cmd = command(N, args, 29500 + i)
        if args.dry_run:
            print(" ".join(cmd))
            continue
        print(f"  HIP-{N:2} GPU...", end=" ", flush=True)
        env = dict(os.environ, MASTER_ADDR="127.0.0.1")
        p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=args.timeout, env=env)
        if p.returncode != 0:
            print(f"FAILED (exit {p.returncode}): {p.stderr.strip().splitlines()[-1:]}")
            continue
        r = last_json(p.stdout)
        why = rejected(r)
        if why:
            print(f"REJECTED ({why})")
            continue
        results.append((N, r))
        print(f"OK ({r['ms_per_step']:.2f} ms, {r['value'] / 1e9:.2f} G suffixes/s)")
    if args.dry_run or not results:
        return 0
    seq = None
    seq_csv = os.path.join(ROOT, "results", "csv", "sequential_results.csv")
    if os.path.exists(seq_csv):
        with open(seq_csv) as f:
            for row in csv.DictReader(f):
                if row.get("file") == workload and row.get("sa_time"):
                    seq = float(row["sa_time"])
    rows = rows_from(results, workload, args.n, seq)
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    with open(args.out, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=COLUMNS)
        w.writeheader()
        w.writerows(rows)
    print("-" * 65)
    print(f"{'File':<25} {'GPU':>5} {'Tempo SA':>10} {'Speedup':>10} {'Efficienza':>12}")
    print("-" * 65)
    for r in rows:
        print(f"{r['file']:<25} {r['processes']:>5} {r['sa_time'] * 1e3:>8.2f}ms {r['speedup']:>9.2f}x "
              f"{r['efficiency'] * 100:>11.1f}%")
    print("-" * 65)
    print(f"Risultati salvati in: {args.out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
