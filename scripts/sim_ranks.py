#!/usr/bin/env python3
"""Per-rank cost of the range-partitioned first round, measured on ONE GPU.

For each world size G the script plays every rank's begin phase in turn
(their coarse histograms summed, i.e. the all_reduce), derives the cuts, and
then times sa_dist_round1 of selected ranks alone on the GPU (HIP events):
what one MI355X of a G-GPU node spends on round 1 of the 1 GiB build before
any collective.  The U rounds (~1 M suffixes at 1 GiB DNA) and the RCCL
collectives are not included.

    python scripts/sim_ranks.py [--n 1073741824] [--kind dna] [--worlds 1,2,4,8] [--reps 5]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 30)
    ap.add_argument("--kind", default="dna")
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    import torch

    from bench import ALPHABETS
    from hpc_suffix_array_amd.distributed import HipRangeOps
    dev = torch.device("cuda", 0)
    ops = HipRangeOps(0, 0)
    n = a.n
    text = torch.empty(n, dtype=torch.uint8, device=dev)
    ops.b.generate_text(text, n, ALPHABETS[a.kind], seed=1)
    present = ops.alphabet(text)
    out = []
    for G in (int(x) for x in a.worlds.split(",")):
        total = torch.zeros(4096, dtype=torch.int64, device=dev)
        for q in range(G):
            info, coarse = ops.begin(text, n, G, q, present)
            if G > 1:
                total += coarse
        ch = total.cpu() if G > 1 else None
        for q in sorted({0, G // 2, G - 1}):
            ops.begin(text, n, G, q, present)
            info = ops.cuts(ch)
            sa_local = torch.empty(info["m"], dtype=torch.int32, device=dev)
            ts = []
            for _ in range(a.reps + 1):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                r1 = ops.round1(sa_local)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            ts = sorted(ts[1:])
            row = {"world": G, "rank": q, "m": info["m"], "share": round(info["m"] / (n / G), 4),
                   "round1_ms": round(ts[len(ts) // 2], 3), "unsorted": r1["unsorted"], "ok": r1["round1_ok"]}
            print(json.dumps(row), flush=True)
            out.append(row)
            del sa_local
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
