#!/usr/bin/env python3
"""A/B of debug-flag variants of one build in ONE process (one workspace,
so no allocation-mode difference between the variants): the 1 GiB text is
built `reps` times per variant, interleaved, with per-kernel HIP events;
prints the median ms per kernel kind.

    python scripts/ab_debug.py [--n N] [--kind dna] [--reps 6] default no_xq ...
(variant "default" = no debug flags; "a+b" = several flags; a part
"t:<int>" sets sa_opts.tune instead, e.g. t:0x20000 = local-sort variant 1)"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 30)
    ap.add_argument("--kind", default="dna")
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--schedule", default="packed", choices=["packed", "reference"])
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    import torch

    from bench import ALPHABETS
    from hpc_suffix_array_amd import DeviceBuilder
    b = DeviceBuilder(a.n)
    t = torch.empty(a.n, dtype=torch.uint8, device="cuda")
    if a.kind == "degenerate":
        t.fill_(ord("a"))
    else:
        b.generate_text(t, a.n, ALPHABETS[a.kind], seed=1)
    sa = torch.empty(a.n, dtype=torch.int32, device="cuda")
    def opts(v):
        parts = [] if v == "default" else v.split("+")
        tune = sum(int(p[2:], 0) for p in parts if p.startswith("t:"))
        return tuple(p for p in parts if not p.startswith("t:")), tune

    res = {v: [] for v in a.variants}
    ok = {}
    for v in a.variants:   # warm-up, and every variant's SA checked
        dbg, tune = opts(v)
        b.build(t, a.n, sa, profile=True, schedule=a.schedule, debug=dbg, tune=tune)
        ok[v] = b.check(t, a.n, sa)
    for _ in range(a.reps):
        for v in a.variants:
            dbg, tune = opts(v)
            torch.cuda.synchronize()
            st = b.build(t, a.n, sa, profile=True, schedule=a.schedule, debug=dbg, tune=tune)
            torch.cuda.synchronize()
            res[v].append(st)
    for v, sts in res.items():
        kinds = [k for k, x in sts[0]["kernels"].items() if x["launches"]]
        med = {k: statistics.median(s["kernels"][k]["ms"] for s in sts) for k in kinds}
        tot = statistics.median(s["total_ms"] for s in sts)
        rounds = [round(statistics.median(s["round_ms"][j] for s in sts), 3) for j in range(sts[-1]["rounds"])]
        print(f"{v:14s} total {tot:7.3f} " + " ".join(f"{k} {x:.3f}" for k, x in med.items())
              + f" rounds {rounds} layout {sts[-1].get('round1_layout')}", flush=True)
    print("checked", ok)
    b.close()


if __name__ == "__main__":
    main()
