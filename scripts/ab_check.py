#!/usr/bin/env python3
"""A/B of the O(n) checker's variants (sa_check.h; sa_context_set_debug tune
bits 20-23: 0 = 256 level-1 bins, 1 = 1024, 2 = 512, 3 = the persistent
prefetching level 2, k_split_p) and the LCP, in ONE
process on one 1 GiB build: interleaved, median ms per variant.

    python scripts/ab_check.py [--n N] [--kind dna] [--reps 5] 0 1 2"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 30)
    ap.add_argument("--kind", default="dna")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("variants", nargs="+", type=int)
    a = ap.parse_args()
    import torch

    from bench import ALPHABETS
    from hpc_suffix_array_amd import DeviceBuilder
    b = DeviceBuilder(a.n)
    t = torch.empty(a.n, dtype=torch.uint8, device="cuda")
    b.generate_text(t, a.n, ALPHABETS[a.kind], seed=1)
    sa = torch.empty(a.n, dtype=torch.int32, device="cuda")
    b.build(t, a.n, sa)
    lcp = torch.empty(a.n, dtype=torch.int32, device="cuda")
    res = {v: [] for v in a.variants}
    lres = {v: [] for v in a.variants}
    for r in range(a.reps + 1):
        for v in a.variants:
            b.set_debug(tune=v << 20)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ok = b.check(t, a.n, sa)
            t1 = time.perf_counter()
            b.lcp(t, a.n, sa, lcp)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            assert ok, v
            if r:
                res[v].append(1e3 * (t1 - t0))
                lres[v].append(1e3 * (t2 - t1))
    for v in a.variants:
        print(f"variant {v}: check {statistics.median(res[v]):.3f} ms  lcp {statistics.median(lres[v]):.3f} ms", flush=True)
    # a corrupted SA must fail under every variant
    sa[[5, 6]] = sa[[6, 5]]
    for v in a.variants:
        b.set_debug(tune=v << 20)
        assert not b.check(t, a.n, sa), v
    print("corruption detected by every variant")
    b.close()


if __name__ == "__main__":
    main()
