#!/usr/bin/env python3
"""Pass-to-pass timing modes: several DeviceBuilders in one process (fresh
context buffers each), optionally with a pad allocation in between, 1 GiB
DNA; prints the per-kernel HIP-event ms of each builder (median of reps)."""
import statistics
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from bench import ALPHABETS
    from hpc_suffix_array_amd import DeviceBuilder
    n = 1 << 30
    dev = torch.device("cuda", 0)
    text = torch.empty(n, dtype=torch.uint8, device=dev)
    sa = torch.empty(n, dtype=torch.int32, device=dev)
    pads = []
    for k in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
        b = DeviceBuilder(n)
        if k == 0:
            b.generate_text(text, n, ALPHABETS["dna"], seed=1)
        rows = []
        for _ in range(4):
            st = b.build(text, n, sa, profile=True)
            torch.cuda.synchronize()
            rows.append(st)
        ks = rows[-1]["kernels"]
        med = {name: statistics.median(r["kernels"][name]["ms"] for r in rows[1:]) for name in
               ("scatter_first", "scatter_keys", "local_sort") if name in ks}
        print(k, {a: round(v, 3) for a, v in med.items()}, round(statistics.median(r["total_ms"] for r in rows[1:]), 3),
              flush=True)
        b.close()
        pads.append(torch.empty((k + 1) * (3 << 20) + 4096 * 7, dtype=torch.uint8, device=dev))


if __name__ == "__main__":
    main()
