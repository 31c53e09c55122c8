#!/usr/bin/env python3
"""Per-rank first round of the range-partitioned build, played on ONE GPU.

For a world size G the script plays every rank's begin phase in turn (their
coarse histograms summed: the all_reduce), derives each rank's cut (the same
plan on every rank), then runs sa_dist_round1 of the selected ranks one
after the other on the GPU (HIP events): what one MI355X of a G-GPU node
spends on round 1 before any collective.  The later doubling rounds (rank
look-ups across ranks by all_to_all) and the RCCL collectives are not
played.

--check verifies, for every rank (configs[3]: byte256 at n = 2^32, G = 8 --
a shape no single GPU builds end to end, replacing manber_myers_mpi.c:47-49's
block split and the root sort of :108-144):
  * the ranks' ranges tile the text's suffixes: sum of m_q = n, and every
    position lands in exactly one rank's round-1 SA slice (a count per
    position, all ones at the end);
  * each slice is sorted on the first K symbols (end of text smallest), and
    the slices follow each other in SA order (the last K-prefix of rank q <=
    the first of rank q + 1; sa_off_q + m_q = sa_off_{q+1}).

    python scripts/sim_ranks.py [--n 1073741824] [--kind dna] [--worlds 1,2,4,8] [--reps 5]
    python scripts/sim_ranks.py --n 4294967296 --kind byte256 --worlds 8 --all-ranks --check --reps 1
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CHUNK = 1 << 25   # torch elementwise / index ops over slices of at most this many elements


def prefix_keys(torch, text, n, sa, K):
    """int64 key of the first K symbols of each suffix sa[i] (K <= 7): digits
    byte + 1 in base 257, 0 past the end, so key order = the order of the
    K-prefixes with the end smallest (equal keys: equal K-prefixes)."""
    assert K <= 7, "257^K must fit int64"
    pos = sa.to(torch.int64) & 0xFFFFFFFF
    key = torch.zeros(pos.numel(), dtype=torch.int64, device=pos.device)
    for t in range(K):
        p = pos + t
        inside = p < n
        d = torch.where(inside, text[torch.where(inside, p, 0)].to(torch.int64) + 1, 0)
        key = key * 257 + d
    return key


def check_rank(torch, text, n, sa_local, K, flags):
    """Sortedness of one rank's slice on its first K symbols, its positions
    counted in flags (int32 per text position); returns (first, last) key."""
    m = sa_local.numel()
    first = last = None
    prev = None
    for a in range(0, m, CHUNK):
        k = prefix_keys(torch, text, n, sa_local[a: a + CHUNK], K)
        if k.numel() > 1:
            assert bool((k[1:] >= k[:-1]).all()), f"slice not sorted on its first {K} symbols near {a}"
        if prev is not None:
            assert int(k[0]) >= prev, f"slice not sorted across {a}"
        prev = int(k[-1])
        if first is None:
            first = int(k[0])
        last = prev
        pos = sa_local[a: a + CHUNK].to(torch.int64) & 0xFFFFFFFF
        flags.index_put_((pos,), torch.ones_like(pos, dtype=flags.dtype), accumulate=True)
    return first, last


def simulate(n, kind, worlds, ranks="ends", reps=5, check=False, seed=1, log=print):
    import torch

    from bench import ALPHABETS
    from hpc_suffix_array_amd.distributed import HipRangeOps
    dev = torch.device("cuda", 0)
    ops = HipRangeOps(0, 0)
    text = torch.empty(n, dtype=torch.uint8, device=dev)
    ops.b.generate_text(text, n, ALPHABETS[kind], seed=seed)
    present = ops.alphabet(text)
    out = []
    for G in worlds:
        total = torch.zeros(4096, dtype=torch.int64, device=dev)
        for q in range(G):
            info, coarse = ops.begin(text, n, G, q, present)
            assert info["status"] == 0, f"no bucketed plan for {kind} n={n} G={G}: {info}"
            if G > 1:
                total += coarse
        ch = total.cpu() if G > 1 else None
        plan = []
        for q in range(G):   # every rank's cut (the same plan everywhere)
            ops.begin(text, n, G, q, present)
            plan.append(ops.cuts(ch))
        assert all(p["status"] == 0 for p in plan), f"cut plan unbalanced: {[p['m'] for p in plan]}"
        if check:
            assert sum(p["m"] for p in plan) == n, "the ranks' ranges do not cover n suffixes"
            for q in range(G - 1):
                assert plan[q]["sa_off"] + plan[q]["m"] == plan[q + 1]["sa_off"], "ranges not contiguous"
                assert plan[q]["bucket_hi"] == plan[q + 1]["bucket_lo"] or G == 1
        sel = range(G) if ranks == "all" else sorted({0, G // 2, G - 1})
        flags = torch.zeros(n, dtype=torch.int32, device=dev) if check else None
        ends = {}
        for q in sel:
            ops.begin(text, n, G, q, present)
            info = ops.cuts(ch)
            sa_local = torch.empty(info["m"], dtype=torch.int32, device=dev)
            ts = []
            for _ in range(reps + 1):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                r1 = ops.round1(sa_local)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            ts = sorted(ts[1:]) if len(ts) > 1 else ts
            row = {"world": G, "rank": q, "n": n, "kind": kind, "m": info["m"], "sa_off": info["sa_off"],
                   "share": round(info["m"] / (n / G), 4), "K": info["K"], "bucket_bits": info["bucket_bits"],
                   "round1_ms": round(ts[len(ts) // 2], 3), "unsorted": r1["unsorted"], "ok": r1["round1_ok"]}
            assert r1["round1_ok"] == 1, f"rank {q}: a window exceeded the LDS tile"
            if check:
                ends[q] = check_rank(torch, text, n, sa_local, info["K"], flags)
                row["checked"] = True
            log(json.dumps(row))
            out.append(row)
            del sa_local
            torch.cuda.empty_cache()
        if check and ranks == "all":
            for q in range(G - 1):
                assert ends[q][1] <= ends[q + 1][0], f"rank {q} and {q + 1} overlap in SA order"
            ones = sum(int((flags[a: a + CHUNK] == 1).sum()) for a in range(0, n, CHUNK))
            assert ones == n, "a position is missing from, or repeated across, the slices"
        del flags
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 30)
    ap.add_argument("--kind", default="dna")
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--all-ranks", action="store_true", help="every rank, not only the first, middle and last")
    ap.add_argument("--check", action="store_true", help="verify the partition and the slices' order")
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    out = simulate(a.n, a.kind, [int(x) for x in a.worlds.split(",")], "all" if a.all_ranks else "ends", a.reps,
                   a.check, log=lambda s: print(s, flush=True))
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
