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
    """The first K symbols of each suffix sa[i] as int64 words of up to 7
    symbols each (digits byte + 1 in base 257, 0 past the end): the order of
    the K-prefixes (end smallest) is the lexicographic order of the word
    lists, and equal lists are equal K-prefixes.  Any K (DNA ranges: K = 20)."""
    pos = sa.to(torch.int64) & 0xFFFFFFFF
    words = []
    for t0 in range(0, K, 7):
        key = torch.zeros(pos.numel(), dtype=torch.int64, device=pos.device)
        for t in range(t0, min(K, t0 + 7)):
            p = pos + t
            inside = p < n
            d = torch.where(inside, text[torch.where(inside, p, 0)].to(torch.int64) + 1, 0)
            key = key * 257 + d
        words.append(key)
    return words


def lex_le(a, b):
    """Elementwise a <= b for word lists a, b (lexicographic)."""
    lt = None
    eq = None
    for x, y in zip(a, b):
        l, e = x < y, x == y
        lt = l if lt is None else lt | (eq & l)
        eq = e if eq is None else eq & e
    return lt | eq


def check_rank(torch, text, n, sa_local, K, flags):
    """Sortedness of one rank's slice on its first K symbols, its positions
    counted in flags (int32 per text position); returns (first, last) key
    (tuples of the words)."""
    m = sa_local.numel()
    first = last = None
    prev = None
    for a in range(0, m, CHUNK):
        k = prefix_keys(torch, text, n, sa_local[a: a + CHUNK], K)
        if k[0].numel() > 1:
            assert bool(lex_le([w[:-1] for w in k], [w[1:] for w in k]).all()), \
                f"slice not sorted on its first {K} symbols near {a}"
        head = tuple(int(w[0]) for w in k)
        if prev is not None:
            assert head >= prev, f"slice not sorted across {a}"
        prev = tuple(int(w[-1]) for w in k)
        if first is None:
            first = head
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


def simulate_full(n, kind, G, reps=2, seed=1, log=print, check=True):
    """The whole range-partitioned build of G ranks played on ONE GPU, every
    rank's phases in turn on its own context (G HipRangeOps in this
    process), the collectives played in-process: the count matrix of each
    later round, the requests routed to their owners (what all_to_all moves),
    the answers routed back.  Per rank and round: the HIP-event time of its
    own kernels (as on its own GPU), its unsorted suffixes, the requests it
    sends and how many of them another rank answers (the look-ups that cross
    xGMI: 4 B out + 8 B back each).  One build's SA (all slices) is O(n)-
    checked.  Memory: G contexts of ~90 B per range suffix + one text."""
    import torch

    from bench import ALPHABETS
    from hpc_suffix_array_amd.distributed import HipRangeOps
    dev = torch.device("cuda", 0)
    ops = [HipRangeOps(0, 0) for _ in range(G)]
    text = torch.empty(n, dtype=torch.uint8, device=dev)
    ops[0].b.generate_text(text, n, ALPHABETS[kind], seed=seed)
    torch.cuda.synchronize()

    def timed(fn, *a):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r = fn(*a)
        e1.record()
        e1.synchronize()
        return r, e0.elapsed_time(e1)

    builds = []
    for rep in range(reps + 1):
        words = [0] * 8
        for q in range(G):
            w = ops[q].alphabet(text[n * q // G: n * (q + 1) // G])
            words = [x | y for x, y in zip(words, w)]
        total = torch.zeros(4096, dtype=torch.int64, device=dev)
        for q in range(G):
            info, coarse = ops[q].begin(text, n, G, q, words)
            assert info["status"] == 0, info
            if G > 1:
                total += coarse
        ch = total.cpu() if G > 1 else None
        cut = [ops[q].cuts(ch) for q in range(G)]
        sa = [torch.empty(c["m"], dtype=torch.int32, device=dev) for c in cut]
        rows = [{"rank": q, "m": cut[q]["m"], "sa_off": cut[q]["sa_off"], "round_ms": [], "unsorted": [],
                 "sent": [], "sent_cross": []} for q in range(G)]
        for q in range(G):
            r1, ms = timed(ops[q].round1, sa[q])
            assert r1["round1_ok"] == 1, (q, r1)
            rows[q]["round_ms"].append(ms)
        h = cut[0]["K"]
        exch = []
        req = got = ans = back = None
        while True:
            cnt, ms_c, uns = [], [], []
            for q in range(G):
                (c, info), ms = timed(ops[q].req_count, h, G)
                cnt.append(c)
                ms_c.append(ms)
                uns.append(info["unsorted"])
            if sum(uns) == 0:
                break
            req, ms_f = [], []
            for q in range(G):
                r, ms = timed(ops[q].req_fill, h, sum(cnt[q]))
                req.append(r)
                ms_f.append(ms)
            offs = [[sum(cnt[q][:p]) for p in range(G + 1)] for q in range(G)]
            got = [torch.cat([req[q][offs[q][p]: offs[q][p + 1]] for q in range(G)]) for p in range(G)]
            ans, ms_a = [], []
            for p in range(G):
                a, ms = timed(ops[p].answer, got[p])
                ans.append(a)
                ms_a.append(ms)
            back = []
            for q in range(G):   # answers to q, in the order of q's requests (owner by owner)
                parts = []
                for p in range(G):
                    a0 = sum(cnt[x][p] for x in range(q))
                    parts.append(ans[p][a0: a0 + cnt[q][p]])
                back.append(torch.cat(parts))
            ms_r = []
            for q in range(G):
                _, ms = timed(ops[q].refine, h, back[q], sa[q])
                ms_r.append(ms)
            for q in range(G):
                rows[q]["round_ms"].append(ms_c[q] + ms_f[q] + ms_a[q] + ms_r[q])
                rows[q]["unsorted"].append(uns[q])
                rows[q]["sent"].append(sum(cnt[q]))
                rows[q]["sent_cross"].append(sum(cnt[q][p] for p in range(G) if p != q))
            pair = max((cnt[q][p] for q in range(G) for p in range(G) if p != q), default=0)
            exch.append({"h": h, "requests": sum(sum(c) for c in cnt),
                         "cross": sum(cnt[q][p] for q in range(G) for p in range(G) if p != q),
                         "max_pair_bytes": 12 * pair})
            h *= 2
        builds.append((rows, exch))
        if rep < reps:
            del sa, req, got, ans, back
            torch.cuda.empty_cache()
    rows, exch = builds[-1]
    verified = None
    if check and n <= 0xFFFFFFFF:
        full = torch.cat(sa)
        verified = bool(ops[0].b.check(text, n, full))
        del full
    # per round: the slowest rank's compute (each on its own GPU); medians
    # over the timed builds
    nr = len(rows[0]["round_ms"])
    per_round = []
    for j in range(nr):
        vals = sorted(max(b[0][q]["round_ms"][j] for q in range(G)) for b in builds[1:] or builds)
        per_round.append(round(vals[len(vals) // 2], 3))
    out = {"world": G, "n": n, "kind": kind, "rounds": nr, "verified": verified,
           "m": [r["m"] for r in rows], "share_max": round(max(r["m"] for r in rows) / (n / G), 4),
           "slowest_rank_ms_per_round": per_round, "compute_ms": round(sum(per_round), 3),
           "unsorted_per_round": [sum(r["unsorted"][j] for r in rows) for j in range(nr - 1)],
           "requests_per_round": [e["requests"] for e in exch],
           "cross_requests_per_round": [e["cross"] for e in exch],
           "xgmi_bytes_per_round": [12 * e["cross"] for e in exch],
           "max_pair_bytes_per_round": [e["max_pair_bytes"] for e in exch],
           "per_rank_round1_ms": [round(r["round_ms"][0], 3) for r in rows]}
    log(json.dumps(out))
    for o in ops:
        o.b.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 30)
    ap.add_argument("--kind", default="dna")
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--all-ranks", action="store_true", help="every rank, not only the first, middle and last")
    ap.add_argument("--check", action="store_true", help="verify the partition and the slices' order")
    ap.add_argument("--full", action="store_true",
                    help="play the whole build (later rounds and their exchanges) of every rank per world size")
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()
    if a.full:
        out = [simulate_full(a.n, a.kind, int(G), max(a.reps, 1), log=lambda s: print(s, flush=True))
               for G in a.worlds.split(",")]
        if a.json_out:
            with open(a.json_out, "w") as f:
                json.dump(out, f, indent=1)
        return
    out = simulate(a.n, a.kind, [int(x) for x in a.worlds.split(",")], "all" if a.all_ranks else "ends", a.reps,
                   a.check, log=lambda s: print(s, flush=True))
    if a.json_out:
        with open(a.json_out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
