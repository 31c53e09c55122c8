#!/usr/bin/env python3
"""bench.py -- suffixes sorted/s + ms per doubling round on MI355X.

BASELINE.json metric: "suffixes sorted/sec + ms/doubling-round, 1 GiB input
at 1/2/4/8 MI355X".  Workload (configs[2]): 1 GiB (n = 2^30) random DNA,
seeded splitmix64, generated directly in HBM.  One step =
one complete suffix-array construction (every doubling round: radix passes,
re-rank, read-backs) from text resident in HBM to SA resident in HBM.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n N] [--kind dna]

N = 1: the single-GPU builder (libsa_hip sa_build_device); "scaling":
"strong" (the 1-GPU point of the strong-scaling curve).
N > 1 (launched by torch.distributed.run, one process per GPU, RCCL): by
default the range-partitioned build of ONE n-symbol string over all ranks
(hpc_suffix_array_amd/distributed.py) -- total work fixed, "scaling":
"strong"; `--mode replicas` instead builds one string per rank (weak).

Output: one JSON line on rank 0 with the driver's contract keys plus
"roofline" (the dominant kernel -- most HIP-event time per build -- with its
algorithmic bytes per launch over its mean launch duration, timed in the
timed region; N = 1; "traffic" from the committed rocprof summary of the same
workload), "kernels_gbs" (the same for every kernel kind) and "cpu_baseline"
(the oracle's reference-identical single-thread restatement of src/sequential
on a bounded sample, rank 0, N = 1 only) and "reference_schedule" (N = 1: the
same text built with the north-star schedule -- one LSD-sorted doubling round
per h, manber_myers.c:97-125 -- so its ms/doubling-round compares with the
reference's rounds; not the headline value).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import re
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
from hpc_suffix_array_amd._native import source_hash   # noqa: E402  (no GPU, no torch)
SRC_HASH = source_hash()
METRIC = "suffixes sorted/sec + ms/doubling-round, 1 GiB input at 1/2/4/8 MI355X"   # BASELINE.json metric

ALPHABETS = {
    "dna": b"ACGT",
    # string.ascii_letters + string.digits (generate_large_datasets.py:14)
    "alnum": b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789",
    "ascii127": bytes(range(1, 128)),
    "byte256": bytes(range(256)),
}


# bench kernel kind -> the HIP kernel it times (sa_build.hip Timer kinds)
KERNEL_NAMES = {
    "scatter_keys": "k_split_seg<SrcPk8,9,12> (second bucket pass over packed 8-byte items; SrcBucketKeys,9,10 "
                    "over key1 + position when they do not fit: units cut at the first pass's digit segments, places "
                    "by per-(low, high digit) cursors, no look-back) | k_onesweep<SrcKeys,1024,4> (LSD first round)",
    "scatter_first": "k_split_text<12,1024,POW2,PK8> (first bucket pass: key1 from the text, packed 8-byte items "
                     "scattered by atomic cursors) | k_onesweep<SrcKeysIota,1024,4> (LSD first round)",
    "local_sort": "k_bucket_sort<512,18> (per-window LDS sort: counting scatter + register sorting networks, "
                  "largest sub-bucket first; SA written; every 16th key1 too only where a later round searches it)",
    "pack": "k_bucket_hist (first-pass digit totals) | k_pack_text (LSD first round keys)",
    "seg_count": "k_seg_count", "seg_write": "k_seg_write | k_wscan_* + k_u_gather",
    "sort_u": "unsorted-set sorts (k_materialize + k_onesweep<SrcKeys>)",
    "pivot_keys": "k_pivot_keys (pivot round keys g << wr | rank[i + h], group starts)",
    "pivot_count": "k_pivot_pass<0> + k_scan_rows (pivot round class counts)",
    "pivot_write": "k_pivot_pass<3> (pivot round: tied blocks to the next unsorted set, the rest compacted)",
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
    ap.add_argument("--cpu-sample-n", type=int, default=1 << 26)
    ap.add_argument("--no-reference-schedule", action="store_true",
                    help="skip the companion build with the north-star schedule (N = 1, packed runs only)")
    ap.add_argument("--no-profile", action="store_true", help="no per-launch HIP events")
    ap.add_argument("--no-lcp", action="store_true",
                    help="skip the timed LCP + O(n) check after the build (N = 1: post_build)")
    ap.add_argument("--schedule", default="packed", choices=["packed", "reference"])
    ap.add_argument("--init-chars", type=int, default=0)
    ap.add_argument("--radix", default="onesweep", choices=["onesweep", "reduce_scan"])
    ap.add_argument("--round1", default="auto", choices=["auto", "lsd", "bucketed"])
    ap.add_argument("--mode", default=None, choices=["distributed", "replicas"],
                    help="distributed (default for N > 1): one string range-partitioned over all ranks (strong "
                         "scaling; --mode distributed also runs the distributed driver at N = 1); replicas: one "
                         "string per rank (weak scaling, opt-in)")
    ap.add_argument("--json-out", default=None)
    return ap.parse_args()


def cpu_baseline(kind: str, n_sample: int, seed: int, reps: int = 3) -> dict:
    """Reference-identical CPU restatement (oracle/mm_oracle.c = the two-pass
    counting sort of manber_myers.c:15-133), one thread pinned to one core
    (`taskset -c 0`; here sched_setaffinity of this process
    around the timing), SA_TIME semantics (build only; create is a memcpy),
    median of `reps`."""
    from oracle import oracle as O
    O.build_oracle()
    t = O.gen_text(kind if kind != "degenerate" else "degenerate", n_sample, seed=seed)
    times, rounds = [], 0
    old = os.sched_getaffinity(0) if hasattr(os, "sched_getaffinity") else None
    core = min(old) if old else None
    try:
        if core is not None:
            os.sched_setaffinity(0, {core})
        for _ in range(reps):
            t0 = time.perf_counter()
            _, rounds, _, _ = O.sa_c(t, stats=True)
            times.append(time.perf_counter() - t0)
    finally:
        if old is not None:
            os.sched_setaffinity(0, old)
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
    out = {"value": n_sample / med, "unit": "suffixes/s", "cores": 1, "kind": "port",
           "sample": f"{kind} n={n_sample} seed={seed}, oracle/mm_oracle.c single thread pinned to core {core}, "
                     f"median of {reps} ({med:.2f} s, {rounds} rounds), cpu '{model}', "
                     f"host cpus {os.cpu_count()}"}
    # the same restatement at configs[2]'s full size, timed once on a GPU box
    # host (scripts/cpu_baseline_1g.py; ~150 s, so not inside every bench run)
    full = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r06_cpu_baseline_1g.txt")
    if kind == "dna" and os.path.exists(full):
        for line in open(full):
            if line.startswith("{"):
                f = json.loads(line)
                out["full_size"] = {"n": f["n"], "value": f["suffixes_per_s"], "seconds": f["seconds"],
                                    "cores": f["cores"], "cpu": f["cpu"],
                                    "sa_matches_known_answer": f["sa_sha256_matches_known_answer"],
                                    "source": "profiles/r06_cpu_baseline_1g.txt"}
    return out


def tag_order(tag: str) -> tuple:
    """Sort key of a profile tag: round, then the version within the round.
    Round 1 used v<number> (r01_v9 < r01_v30), later rounds letter tags in
    bijective base 26 (r02_o < r02_z < r02_aa < r02_bb): length, then text."""
    m = re.match(r"r(\d+)_(.+)$", tag)
    if not m:
        return (-1, 0, 0, tag)
    rnd, rest = int(m.group(1)), m.group(2)
    v = re.fullmatch(r"v(\d+)", rest)
    if v:
        return (rnd, 0, int(v.group(1)), "")
    return (rnd, 1, len(rest), rest)


def pmc_summary(n: int, kind: str, src_hash: str | None, profiles_dir: str | None = None) -> dict | None:
    """The rocprofv3 summary (profiles/<tag>_summary.json, written by
    profiles/collect.sh + summarize.py) of this workload: among the summaries
    of the same n and kind, the one stamped with the current sources' hash
    (latest tag if several); else the latest one, marked "stale" (its
    traffic measured older code).  None when no summary has this workload."""
    d = profiles_dir or os.path.join(ROOT, "profiles")
    cands = []
    for p in glob.glob(os.path.join(d, "*_summary.json")):
        try:
            with open(p) as f:
                s = json.load(f)
        except (OSError, ValueError):
            continue
        args = list(s.get("args") or [])
        extra = [x for i, x in enumerate(args) if x not in ("--n", "--kind") and (i == 0 or args[i - 1] not in ("--n", "--kind"))]
        if s.get("n") == n and s.get("kind") == kind and not extra:
            tag = s.get("tag") or os.path.basename(p)[: -len("_summary.json")]
            cands.append((tag_order(tag), tag, s))
    if not cands:
        return None
    cands.sort(key=lambda x: x[0])
    same = [c for c in cands if src_hash and c[2].get("src_hash") == src_hash]
    _, tag, s = (same or cands)[-1]
    return dict(s, tag=tag, stale=not same)


def make_text(b, n, kind, seed, dev, sptr):
    import torch
    d_text = torch.empty(n, dtype=torch.uint8, device=dev)
    if kind == "degenerate":
        d_text.fill_(ord("a"))
    else:
        b.generate_text(d_text, n, ALPHABETS[kind], seed=seed, stream=sptr)
    return d_text


def timed(steps, warmup, fn, barrier):
    for _ in range(warmup):
        fn()
    barrier()
    t0 = time.perf_counter()
    res = [fn() for _ in range(steps)]
    barrier()
    return time.perf_counter() - t0, res


def reference_schedule(b, d_text, n, d_sa, sptr, a, torch, dev, reps: int = 2) -> dict:
    """The north-star-shaped schedule beside the packed headline: one
    doubling round per h = 1, 2, 4, ... (manber_myers.c:97-125), each a
    full LSD radix sort of (rank, rank[i+h]) keys.  One warm-up build, then
    `reps` timed builds (wall clock between stream syncs), and the O(n)
    check of the last one -- not part of the headline `value`."""
    kw = dict(stream=sptr, profile=True, schedule="reference", init_chars=0, radix=a.radix)
    b.build(d_text, n, d_sa, **kw)
    times, st = [], None
    for _ in range(reps):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        st = b.build(d_text, n, d_sa, **kw)
        torch.cuda.synchronize(dev)
        times.append(time.perf_counter() - t0)
    ms = 1e3 * statistics.median(times)
    return {"ms_per_step": round(ms, 3), "value": n / (ms / 1e3), "rounds": st["rounds"],
            "ms_per_round": [round(x, 3) for x in st["round_ms"]], "prefix_len_per_round": st["prefix_len"],
            "passes_per_round": st["passes"], "distinct_per_round": st["distinct"],
            "roofline_per_round": model_rounds(n, st["distinct"], st["round_ms"]),
            "kernels_ms": {k: round(v["ms"], 3) for k, v in st["kernels"].items() if v["launches"]},
            "verified": b.check(d_text, n, d_sa, stream=sptr)}


def post_build(b, d_text, n, d_sa, sptr, torch, dev, reps: int = 3) -> dict:
    """The reference caller's flow after build_suffix_array
    (main_sequential.c:108-120): build_lcp_array + the longest repeated
    substring (LCP_TIME, manber_myers.c:135-182) and is_valid_suffix_array
    (:184-202), each on the GPU from the SA in HBM: one warm-up, then the
    median wall time of `reps` (stream-synchronised) calls.  Not part of the
    headline `value`."""
    d_lcp = torch.empty(n, dtype=torch.int32, device=dev)

    def clock(fn):
        fn()
        ts, res = [], None
        for _ in range(reps):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            res = fn()
            torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - t0)
        return 1e3 * statistics.median(ts), res

    lcp_ms, (lrs_len, lrs_pos) = clock(lambda: b.lcp(d_text, n, d_sa, d_lcp, stream=sptr))
    check_ms, ok = clock(lambda: b.check(d_text, n, d_sa, stream=sptr))
    del d_lcp
    return {"lcp_ms": round(lcp_ms, 3), "lrs_len": lrs_len, "lrs_sa_pos": lrs_pos,
            "check_ms": round(check_ms, 3), "check_ok": ok,
            "check_bytes_per_suffix": 77,
            "check_gbs": round(77 * n / (check_ms / 1e3) / 1e9, 1) if check_ms > 0 else None}


def model_rounds(n: int, distinct, round_ms) -> list:
    """SURVEY.md 8(d)'s per-round model against the measured round times:
    B_j = n (3 rb + 2 S (P_j + 1)), P_j = ceil(2 w_j / 8), w_j = bit width
    of D_{j-1} with D_0 = 256 (manber_myers.c:94), rb = 4, S = 12 below 2^31
    (8 / 24 above); frac = B_j / t_j / the 8 TB/s HBM peak."""
    rb, S = (4, 12) if n < (1 << 31) else (8, 24)
    out, prev = [], 256
    for d, ms in zip(distinct, round_ms):
        P = -(-2 * int(prev).bit_length() // 8)
        B = n * (3 * rb + 2 * S * (P + 1))
        gbs = B / (ms / 1e3) / 1e9 if ms > 0 else None
        out.append({"P_model": P, "model_bytes": B, "ms": round(ms, 3), "gbs": gbs and round(gbs, 1),
                    "frac": gbs and round(gbs / HBM_PEAK_GBS, 4)})
        prev = d
    return out


def run_single(a, torch, dev, world, rank, barrier):
    """Single-GPU builder; with world > 1 (--mode replicas) one string per rank."""
    from hpc_suffix_array_amd import DeviceBuilder
    n = a.n
    b = DeviceBuilder(n, device=dev.index)
    sptr = torch.cuda.current_stream(dev).cuda_stream
    d_text = make_text(b, n, a.kind, a.seed + rank, dev, sptr)
    d_sa = torch.empty(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize(dev)
    profile = not a.no_profile
    bkw = dict(stream=sptr, profile=profile, schedule=a.schedule, init_chars=a.init_chars, radix=a.radix,
               round1=a.round1)
    elapsed, stats = timed(a.steps, a.warmup, lambda: b.build(d_text, n, d_sa, **bkw), barrier)
    verified = b.check(d_text, n, d_sa, stream=sptr)
    post = post_build(b, d_text, n, d_sa, sptr, torch, dev) if (world == 1 and not a.no_lcp) else None
    ref_sched = None
    if world == 1 and a.schedule == "packed" and not a.no_reference_schedule:
        ref_sched = reference_schedule(b, d_text, n, d_sa, sptr, a, torch, dev)

    rounds = stats[-1]["rounds"]
    round_ms = [statistics.mean(s["round_ms"][j] for s in stats) for j in range(rounds)]
    kern = {}
    for k in stats[-1]["kernels"]:
        kern[k] = {key: sum(s["kernels"][k][key] for s in stats) for key in ("ms", "launches", "bytes")}
    bucketed = stats[-1].get("round1") == "bucketed"
    roofline = None
    per_kernel = None
    if profile:
        # achieved GB/s of every kind: algorithmic bytes per launch / mean
        # HIP-event duration of its launches (all on the build's stream)
        per_kernel = {}
        for k, v in kern.items():
            if v["launches"] and v["ms"] > 0 and v["bytes"]:
                per_kernel[k] = {"ms_per_step": round(v["ms"] / a.steps, 3), "launches_per_step": v["launches"] / a.steps,
                                 "gbs": round(v["bytes"] / (v["ms"] / 1e3) / 1e9, 1)}
        # the dominant kernel: most time per step
        cand = {k: v for k, v in kern.items() if k not in ("scan",) and v["launches"] and v["bytes"]}
        dom = max(cand, key=lambda k: cand[k]["ms"]) if cand else None
        if dom:
            avg_s = kern[dom]["ms"] / kern[dom]["launches"] / 1e3
            per_launch = kern[dom]["bytes"] / kern[dom]["launches"]
            ach = per_launch / avg_s / 1e9
            traffic = traffic_src = None
            pmc = pmc_summary(n, a.kind, SRC_HASH)
            if pmc:
                skind = {"scatter_first": "scatter_first" if bucketed else "scatter_iota"}.get(dom, dom)
                traffic = pmc.get("traffic_bytes_per_launch", {}).get(skind)
                traffic_src = {"summary": f"profiles/{pmc['tag']}_summary.json", "src_hash": pmc.get("src_hash"),
                               "stale": pmc["stale"]}
            roofline = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                        "kernel": KERNEL_NAMES.get(dom, dom) + (" [bucketed round 1]" if bucketed else ""),
                        "kind": dom, "bytes_per_launch": int(per_launch), "avg_launch_ms": round(avg_s * 1e3, 4)}
    # SURVEY.md 8(d)'s whole-build figure: the algorithmic bytes of every
    # kernel of one build over the build's wall time (t_SA), beside the
    # dominant kernel's roofline
    build_bytes = sum(v["bytes"] for v in kern.values()) / a.steps
    t_sa = elapsed / a.steps
    build_roofline = None
    if build_bytes and t_sa > 0:
        ach_b = build_bytes / t_sa / 1e9
        build_roofline = {"bound": "hbm", "achieved": round(ach_b, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(ach_b / HBM_PEAK_GBS, 4), "bytes_per_build": int(build_bytes),
                          "bytes_per_suffix": round(build_bytes / n, 2), "t_sa_ms": round(1e3 * t_sa, 3)}
    extra = {
        "build_roofline": build_roofline,
        # the packed schedule's rounds: round 1 sorts by the first K symbols
        # at once (the reference's rounds h = 1 .. K/2), so these are not per
        # doubling; ms_per_doubling_round is the reference schedule's
        "ms_per_packed_round": [round(x, 3) for x in round_ms],
        "rounds": rounds,
        "distinct_per_round": stats[-1]["distinct"],
        "passes_per_round": stats[-1]["passes"],
        "sorted_per_round": stats[-1]["sorted_n"],
        "prefix_len_per_round": stats[-1]["prefix_len"],
        "schedule": stats[-1]["schedule"],
        "init_chars": stats[-1]["init_chars"],
        "sigma": stats[-1]["sigma"],
        "sparse_ranks": stats[-1]["sparse_ranks"],
        # SURVEY.md 8(d)'s byte model of the REFERENCE-shaped schedule (12-B
        # records through P_j LSD passes per round) for this text: what the
        # reference's algorithm would move, NOT the bytes of the packed
        # schedule measured here (bytes_per_packed_round / build_roofline)
        "reference_model_bytes": stats[-1]["reference_model_bytes"],
        # the packed schedule's own algorithmic bytes per round (the kernels
        # launched between the round's boundaries) and their rate over the
        # round's HIP-event time
        "bytes_per_packed_round": stats[-1]["round_bytes"],
        "gbs_per_packed_round": [round(b / (ms / 1e3) / 1e9, 1) if ms > 0 else None
                                 for b, ms in zip(stats[-1]["round_bytes"], round_ms)],
        "round1": stats[-1].get("round1"),
        "largest_window": stats[-1].get("largest_window"),
        "verified": verified,
        "roofline": roofline,
        "kernels_gbs": per_kernel,
        "kernels_ms_per_step": {k: round(v["ms"] / a.steps, 3) for k, v in kern.items()} if profile else None,
        "reference_schedule": ref_sched,
        # the calls every reference caller makes after the build
        # (main_sequential.c:108-120), timed outside `value`
        "post_build": post,
        # the packed schedule's round 1 covers the reference's rounds h = 1 ..
        # K/2 at once, so its ms_per_round are not per doubling: the build's
        # time over the reference's own round count for this text
        # (manber_myers.c:97-125, the companion schedule's rounds)
        "ms_per_reference_round": (round(1e3 * elapsed / a.steps / ref_sched["rounds"], 3)
                                   if ref_sched and ref_sched.get("rounds") else None),
        # ms per doubling round as the metric reads it (manber_myers.c:97-125):
        # the north-star schedule's measured rounds, one LSD sort per h
        "ms_per_doubling_round": ref_sched["ms_per_round"] if ref_sched else None,
    }
    b.close()
    return elapsed, extra


XGMI_BYTES_PER_REQUEST = 4 + 8   # a request is a u32 position, its answer an i64 rank (distributed.py)


def rank_record(rank: int, stats: list, round1_kernels: dict | None) -> dict:
    """One rank's measurements of the timed steps, for distributed_summary:
    its range, the mean HIP-event time of each phase of DistributedSA.build
    and the round-1 kernels of its last build (sa_dist_round1's sa_stats)."""
    st = stats[-1]
    phase = {}
    for x in stats:
        for k, v in (x.get("phase_ms") or {}).items():
            phase[k] = phase.get(k, 0.0) + v / len(stats)
    return {"rank": rank, "m": st.get("m"), "sa_off": st.get("sa_off"), "phase_ms": phase,
            "round1_kernels": round1_kernels or {}, "requests": st.get("requests") or [],
            "cross_requests": st.get("cross_requests") or []}


def distributed_summary(recs: list, n: int) -> dict:
    """The N > 1 line's per-rank figures (every rank's record, rank order):
    - "roofline": the round-1 kernel with the most time on the rank whose
      round 1 is slowest -- its algorithmic bytes per launch (the range's m
      suffixes times the kernel's bytes per suffix, sa_round1.h add_bytes)
      over its mean HIP-event launch duration, against the 8 TB/s peak;
    - "round1_per_rank": each rank's round-1 time, algorithmic bytes and GB/s;
    - "kernels_ms_per_step": each phase's time, max over ranks, and the
      round-1 kernels of the slowest rank;
    - "xgmi_bytes_per_round": the bytes of the rank look-ups answered by
      another rank, per later doubling round (requests out + answers back),
      which cross xGMI under RCCL (look-ups a rank answers itself stay in HBM);
    - "largest_rank_share": the largest range over n / G."""
    G = len(recs)
    per_rank = []
    for r in recs:
        kb = sum(v["bytes"] for v in r["round1_kernels"].values())
        t = r["phase_ms"].get("round1")
        gbs = kb / (t / 1e3) / 1e9 if kb and t else None
        per_rank.append({"rank": r["rank"], "m": r["m"], "round1_ms": t and round(t, 3), "round1_bytes": kb,
                         "gbs": gbs and round(gbs, 1), "frac": gbs and round(gbs / HBM_PEAK_GBS, 4)})
    timed = [x for x in per_rank if x["round1_ms"]]
    slow = max(timed, key=lambda x: x["round1_ms"]) if timed else None
    roofline = None
    if slow:
        kern = recs[slow["rank"]]["round1_kernels"]
        cand = {k: v for k, v in kern.items() if k != "scan" and v["launches"] and v["bytes"] and v["ms"] > 0}
        if cand:
            dom = max(cand, key=lambda k: cand[k]["ms"])
            v = cand[dom]
            per_launch = v["bytes"] / v["launches"]
            avg_s = v["ms"] / v["launches"] / 1e3
            ach = per_launch / avg_s / 1e9
            roofline = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None, "traffic_source": None,
                        "kernel": KERNEL_NAMES.get(dom, dom) + " [range build, round 1]", "kind": dom,
                        "rank": slow["rank"], "bytes_per_launch": int(per_launch),
                        "avg_launch_ms": round(avg_s * 1e3, 4),
                        "scope": "the slowest rank's round-1 kernel with the most time"}
    phases = sorted({k for r in recs for k in r["phase_ms"]})
    kms = {k: round(max(r["phase_ms"].get(k, 0.0) for r in recs), 3) for k in phases}
    if slow:
        kms["round1_kernels_slowest_rank"] = {k: round(v["ms"], 3) for k, v in
                                              recs[slow["rank"]]["round1_kernels"].items() if v["launches"]}
    cross = recs[0]["cross_requests"]
    m_max = max((r["m"] or 0) for r in recs)
    return {"roofline": roofline, "round1_per_rank": per_rank, "kernels_ms_per_step": kms,
            "requests_per_round": recs[0]["requests"], "cross_requests_per_round": cross,
            "xgmi_bytes_per_round": [int(c) * XGMI_BYTES_PER_REQUEST for c in cross],
            "largest_rank_share": round(m_max / (n / G), 4) if m_max else None}


def run_distributed(a, torch, dev, world, rank, barrier):
    """One string over all ranks: the range-partitioned build
    (hpc_suffix_array_amd/distributed.py).  Each rank starts a step from its
    slice of the text only (rank r: text[r C, (r + 1) C), C = n / G), as
    north_star partitions the string; the step gathers the text to every
    rank (one RCCL all_gather, INSIDE the timed step -- the reference times
    its text MPI_Bcast too, main_mpi.c:40-51), then each rank sorts the
    suffixes of its bucket range from its text copy, rank look-ups crossing
    xGMI by RCCL all_to_all between doubling rounds.  Per-phase times are HIP
    events on the build stream."""
    import torch.distributed as dist
    from hpc_suffix_array_amd.distributed import DistributedSA, HipRangeOps, gather_sa, text_chunk
    n = a.n
    # the workspace of a build (range buffers, the gathered text) reserved
    # once, as DeviceBuilder(n) does for one GPU -- not inside the first build
    ops = HipRangeOps(n, dev.index, world=world)
    ops.profile = not a.no_profile   # round 1's per-kernel HIP events (sa_dist_round1 sa_stats)
    sptr = torch.cuda.current_stream(dev).cuda_stream
    C = text_chunk(n, world)
    lo, hi = min(n, rank * C), min(n, (rank + 1) * C)
    # this rank's slice of the seeded text: generated whole (same seed on
    # every rank), sliced, the rest freed -- outside the timed region, as the
    # single-GPU bench's text is generated in HBM before it
    full = torch.empty(n, dtype=torch.uint8, device=dev)
    if a.kind == "degenerate":
        full.fill_(ord("a"))
    else:
        ops.b.generate_text(full, n, ALPHABETS[a.kind], seed=a.seed, stream=sptr)
    d_slice = full[lo:hi].clone()
    del full
    torch.cuda.synchronize(dev)
    holder = {}

    def step():
        d = DistributedSA(ops)
        holder["sa"] = d.build_sliced(d_slice, n)
        torch.cuda.synchronize(dev)
        return d.stats

    elapsed, stats = timed(a.steps, a.warmup, step, barrier)
    r1k = ops.round1_stats.to_dict()["kernels"] if ops.profile and stats[-1].get("path") == "range" else None
    rec = rank_record(rank, stats, r1k)
    recs = [None] * world
    if world > 1:
        dist.all_gather_object(recs, rec)
    else:
        recs = [rec]
    sa_local, sa_off = holder["sa"]
    d_text = ops.textbuf[:n] if world > 1 else d_slice   # the text as the last build gathered it
    # verification: the full SA gathered to every rank, O(n) check on rank 0
    verified = None
    if n <= 0xFFFFFFFF:
        sa = gather_sa(sa_local, sa_off, n)
        if rank == 0:
            verified = ops.b.check(d_text, n, sa.to(torch.int32))
        del sa
    if world > 1:
        v = torch.tensor([1 if verified in (True, None) else 0], dtype=torch.int64, device=dev)
        dist.broadcast(v, 0)
        verified = bool(v.item()) if n <= 0xFFFFFFFF else None
    st = stats[-1]
    summ = distributed_summary(recs, n)
    extra = {"rounds": st["rounds"], "unsorted_per_round": st.get("unsorted"),
             "init_chars": st.get("K"), "sigma": st.get("sigma"), "bucket_bits": st.get("bucket_bits"),
             "path": st.get("path"),
             "phase_ms": {k: round(v, 3) for k, v in rec["phase_ms"].items()},
             # the text all_gather, part of every timed step (phase "text_gather")
             "text_gather_ms": round(rec["phase_ms"].get("text_gather", 0.0), 3) if world > 1 else None,
             "input_partition": f"rank r holds text[r*{C}, (r+1)*{C}) at the start of each step",
             # per build, rank 0: collectives (RCCL calls, each all_to_all
             # slice counted) and host waits (the driver's read-backs and
             # libsa_hip's own stream syncs / blocking copies)
             "collectives_per_build": st.get("collectives"),
             "host_syncs_per_build": st.get("host_syncs"),
             "host_syncs_driver_per_build": st.get("host_syncs_driver"),
             "host_syncs_native_per_build": st.get("host_syncs_native"),
             "verified": verified,
             "note": "range-partitioned build from a range-partitioned string: the text all_gather, then each rank "
                     "sorts the suffixes of its bucket range from its text copy; rank requests/answers by RCCL "
                     "all_to_all between doubling rounds; roofline = the slowest rank's dominant round-1 kernel"}
    extra.update(summ)
    return elapsed, extra


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    use_pg = world > 1 or a.mode == "distributed"
    if use_pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group("nccl", device_id=dev)

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    # N > 1 measures the range-partitioned build of ONE string (strong
    # scaling, BASELINE.json metric at 1/2/4/8 GPUs); replicas are opt-in
    distributed = a.mode == "distributed" or (a.mode is None and world > 1)
    runner = run_distributed if distributed else run_single
    elapsed, extra = runner(a, torch, dev, world, rank, barrier)
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ms_per_step = 1e3 * float(t.item()) / max(a.steps, 1)
    total = a.n if distributed else world * a.n
    out = {
        "metric": METRIC,
        "value": total / (ms_per_step / 1e3),
        "unit": "suffixes/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True,
        "scaling": "weak" if (world > 1 and not distributed) else "strong",
        "vs_baseline": None,
        "dtype": "u32",
        "src_hash": SRC_HASH,
        "data": f"synthetic: seeded splitmix64 {a.kind} text generated in HBM (SURVEY.md 8(d)), seed {a.seed}"
                + ("" if distributed or world == 1 else "+rank"),
        "config": {"workload": f"{a.kind} n={a.n} ({a.n / (1 << 30):.3g} GiB)"
                               + (" over all GPUs" if distributed else " per GPU") + ", full suffix-array build",
                   "n": a.n, "kind": a.kind,
                   "parallelism": (f"range-partitioned x{world}" if distributed
                                   else (f"replicas x{world}" if world > 1 else "single"))},
    }
    out.update(extra)
    out["cpu_baseline"] = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(a.kind, min(a.cpu_sample_n, a.n), a.seed)
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            os.makedirs(os.path.dirname(os.path.abspath(a.json_out)), exist_ok=True)
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if use_pg:
        dist.destroy_process_group()
    # a build that fails the O(n) check must not pass for a measurement
    if out.get("verified") is False or (out.get("reference_schedule") or {}).get("verified") is False:
        print("bench.py: the suffix array failed the O(n) check", file=sys.stderr, flush=True)
        sys.exit(3)


if __name__ == "__main__":
    main()
