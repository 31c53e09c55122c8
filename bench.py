#!/usr/bin/env python3
"""bench.py -- suffixes sorted/s + ms per doubling round on MI355X.

BASELINE.json metric: "suffixes sorted/sec + ms/doubling-round, 1 GiB input
at 1/2/4/8 MI355X".  Workload (configs[2]): 1 GiB (n = 2^30) random DNA,
seeded splitmix64, generated directly in HBM.  One step =
one complete suffix-array construction (every doubling round: radix passes,
re-rank, D_j read-back) from text resident in HBM to SA resident in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n N] [--kind dna]

N > 1 is launched by torch.distributed.run (one process per GPU); in this
round each rank builds the SA of its own 1 GiB string (independent replicas,
weak scaling, no data-path collective -- DESIGN.md "Multi-GPU").

Output: one JSON line on rank 0 with the driver's contract keys plus
"roofline" (dominant kernel: the radix scatter over stored keys, algorithmic
bytes 24 B/suffix per launch, HIP-event timed in the timed region) and
"cpu_baseline" (the oracle's reference-identical single-thread restatement
of src/sequential on a bounded sample, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec

ALPHABETS = {
    "dna": b"ACGT",
    # string.ascii_letters + string.digits (generate_large_datasets.py:14)
    "alnum": b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789",
    "ascii127": bytes(range(1, 128)),
    "byte256": bytes(range(256)),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--n", type=int, default=1 << 30)
    ap.add_argument("--kind", default="dna", choices=sorted(ALPHABETS) + ["degenerate"])
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-n", type=int, default=1 << 25)
    ap.add_argument("--no-profile", action="store_true", help="no per-launch HIP events")
    ap.add_argument("--schedule", default="packed", choices=["packed", "reference"])
    ap.add_argument("--init-chars", type=int, default=0)
    ap.add_argument("--radix", default="onesweep", choices=["onesweep", "reduce_scan"])
    ap.add_argument("--json-out", default=None)
    return ap.parse_args()


def cpu_baseline(kind: str, n_sample: int, seed: int, reps: int = 3) -> dict:
    """Reference-identical CPU restatement (oracle/mm_oracle.c = the two-pass
    counting sort of manber_myers.c:15-133), one thread, SA_TIME semantics
    (build only; create is a memcpy), median of `reps`."""
    from oracle import oracle as O
    O.build_oracle()
    t = O.gen_text(kind if kind != "degenerate" else "degenerate", n_sample, seed=seed)
    times, rounds = [], 0
    for _ in range(reps):
        t0 = time.perf_counter()
        _, rounds, _, _ = O.sa_c(t, stats=True)
        times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": n_sample / med, "unit": "suffixes/s", "cores": 1, "kind": "port",
            "sample": f"{kind} n={n_sample} seed={seed}, oracle/mm_oracle.c single thread, "
                      f"median of {reps} ({med:.2f} s, {rounds} rounds), cpu '{model}'"}


def pmc_traffic() -> dict | None:
    """Per-launch HBM traffic of the dominant kernel from the committed
    rocprofv3 PMC summary (profiles/<tag>_summary.json, written by
    profiles/collect.sh + summarize.py), or None."""
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_summary.json")))
    if not paths:
        return None
    try:
        with open(paths[-1]) as f:
            d = json.load(f)
        return d
    except (OSError, ValueError):
        return None


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    from hpc_suffix_array_amd import DeviceBuilder
    n = a.n
    b = DeviceBuilder(n, device=local)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream
    d_text = torch.empty(n, dtype=torch.uint8, device=dev)
    d_sa = torch.empty(n, dtype=torch.int32, device=dev)
    if a.kind == "degenerate":
        d_text.fill_(ord("a"))
    else:
        b.generate_text(d_text, n, ALPHABETS[a.kind], seed=a.seed + rank, stream=sptr)
    torch.cuda.synchronize(dev)

    profile = not a.no_profile
    bkw = dict(stream=sptr, profile=profile, schedule=a.schedule, init_chars=a.init_chars, radix=a.radix)
    for _ in range(a.warmup):
        b.build(d_text, n, d_sa, **bkw)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    barrier()
    t0 = time.perf_counter()
    stats = []
    for _ in range(a.steps):
        stats.append(b.build(d_text, n, d_sa, **bkw))
    torch.cuda.synchronize(dev)
    barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    ms_per_step = 1e3 * elapsed / max(a.steps, 1)

    verified = b.check(d_text, n, d_sa, stream=sptr)

    # per-round ms (mean over timed steps) and kernel aggregates
    rounds = stats[-1]["rounds"]
    round_ms = [statistics.mean(s["round_ms"][j] for s in stats) for j in range(rounds)]
    kern = {}
    for k in stats[-1]["kernels"]:
        ms = sum(s["kernels"][k]["ms"] for s in stats)
        nl = sum(s["kernels"][k]["launches"] for s in stats)
        by = sum(s["kernels"][k]["bytes"] for s in stats)
        kern[k] = {"ms": ms, "launches": nl, "bytes": by}
    dom = "scatter_keys"
    roofline = None
    if profile and kern[dom]["launches"]:
        avg_s = kern[dom]["ms"] / kern[dom]["launches"] / 1e3
        per_launch = kern[dom]["bytes"] / kern[dom]["launches"]
        ach = per_launch / avg_s / 1e9
        traffic = None
        pmc = pmc_traffic()
        if pmc and pmc.get("n") == n and pmc.get("kind") == a.kind:
            traffic = pmc.get("traffic_bytes_per_launch", {}).get("k_scatter_keys")
        roofline = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                    "kernel": "k_scatter<SrcKeys> (radix downsweep, stored keys)",
                    "bytes_per_launch": int(per_launch), "avg_launch_ms": round(avg_s * 1e3, 4)}

    out = {
        "metric": "suffixes sorted/sec + ms/doubling-round, 1 GiB input",
        "value": world * n / (ms_per_step / 1e3),
        "unit": "suffixes/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": f"synthetic: seeded splitmix64 {a.kind} text generated in HBM (SURVEY.md 8(d)), seed {a.seed}+rank",
        "config": {"workload": f"{a.kind} n={n} ({n / (1 << 30):.3g} GiB) per GPU, full Manber-Myers build",
                   "n": n, "kind": a.kind, "parallelism": f"replicas{world}" if world > 1 else "single"},
        "ms_per_round": [round(x, 3) for x in round_ms],
        "rounds": rounds,
        "distinct_per_round": stats[-1]["distinct"],
        "passes_per_round": stats[-1]["passes"],
        "sorted_per_round": stats[-1]["sorted_n"],
        "prefix_len_per_round": stats[-1]["prefix_len"],
        "schedule": stats[-1]["schedule"],
        "init_chars": stats[-1]["init_chars"],
        "sigma": stats[-1]["sigma"],
        "model_bytes": stats[-1]["model_bytes"],
        "model_frac_of_hbm_peak": round(stats[-1]["model_bytes"] / (ms_per_step / 1e3) / 8e12, 4),
        "verified": verified,
        "roofline": roofline,
        "kernels_ms_per_step": {k: round(v["ms"] / a.steps, 3) for k, v in kern.items()} if profile else None,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(a.kind, min(a.cpu_sample_n, n), a.seed)
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    b.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
