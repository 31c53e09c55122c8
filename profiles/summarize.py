#!/usr/bin/env python3
"""Summarise a profiles/collect.sh run into profiles/<tag>_summary.json.

Per kernel kind: calls, average duration (rocprofv3 kernel trace), FETCH_SIZE
and WRITE_SIZE per launch (rocprofv3 --pmc, KiB -> bytes), and HBM traffic
per launch corrected as MI355X_MICROARCH.md section HBM prescribes: on gfx950
FETCH_SIZE under-reads wide coalesced streams (x2 for 16-B/lane reads) and
other access widths must be calibrated on a known byte count.  The read
calibration here is the k_alphabet launch, which reads exactly the n text
bytes (16 B per lane): read_factor = n / FETCH bytes of that launch (2.0 as
the guide prescribes; the local sort, which reads exactly 12 B per suffix in
8-B and 4-B lanes, lands within 3 % of 12 with the same factor).
WRITE_SIZE is reported as measured (exact for 16-B/lane streaming stores per
the guide; the scatter's 8-B / 4-B run stores are uncalibrated).
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

KINDS = [("k_chk_bin<1024, 8, sa::IsaSrc", "lcp_isa_bin"), ("k_chk_split<1024, 8, 32, 3", "lcp_isa_split"), ("k_perm_split<1024, 8, 32, true, 3", "lcp_isa_split"), ("k_perm_place<1024, false, 3", "lcp_isa_place"), ("k_chk_bin<1024, 8, sa::PlcpSrc", "lcp_place_bin"), ("k_chk_split<1024, 8, 32, 4", "lcp_place_split"), ("k_perm_split<1024, 8, 32, true, 4", "lcp_place_split"), ("k_perm_place<1024, false, 4", "lcp_place_place"), ("k_lcp_best", "lcp_best"), ("k_chk_bin<1024, 8, sa::ChkSrcA", "check_bin_a"), ("k_chk_bin<1024, 8, sa::ChkSrcB", "check_bin_b"),
         ("k_chk_bin<1024, 8, sa::PhiSrc", "lcp_phi_bin"), ("k_chk_split<1024, 8, 32, 2", "lcp_phi_split"),
         ("k_perm_split<1024, 8, 32, true, 2", "lcp_phi_split"), ("k_perm_place<1024, false, 2", "lcp_phi_place"),
         ("k_perm_split<1024, 8, 32, true", "check_split_a"), ("k_perm_split<1024, 8, 40, true", "check_split_b"),
         ("k_chk_split<1024, 8, 32", "check_split_a"), ("k_chk_split<1024, 8, 40", "check_split_b"),
         ("k_perm_place<1024, false, 1", "check_place_a"), ("k_chk_place", "check_place_b"),
         ("k_chk_cursors", "check_small"), ("k_chk_tiles", "check_small"),
         ("k_plcp_irreducible", "lcp_irreducible"), ("k_plcp_long", "lcp_long"),
         ("k_plcp_settle", "lcp_long"), ("k_chunk_max", "lcp_scan"), ("k_scan_chunk_max", "lcp_scan"),
         ("k_plcp_apply", "lcp_scan"), ("k_lcp_gather", "lcp_gather"),
         ("k_pivot_keys", "pivot_keys"), ("k_pivot_pass<0", "pivot_count"), ("k_pivot_pass<1", "pivot_count"), ("k_pivot_pass<2", "pivot_write"),
         ("k_pivot_pass<3", "pivot_write"), ("k_pivot_tied_scan", "pivot_write"),
         ("k_pivot_place", "pivot_place"), ("k_pivot_gp", "pivot_gp"), ("k_lsd_hist", "lsd_hist"),
         ("k_lsd_base", "lsd_base"), ("k_lsd<", "lsd"), ("k_perm_rank", "perm_rank"), ("k_perm_split", "perm_split"),
         ("k_perm_place", "perm_place"), ("k_tile_heads", "heads"), ("k_items_to_sa", "items_to_sa"),
         ("k_split_list", "scatter_first"), ("k_usort_small", "sort_u_small"), ("k_usort_keys", "sort_u_keys"),
         ("k_bucket_sample", "pack"), ("k_window_split", "windows"), ("k_window_list", "windows"),
         ("k_split_text", "scatter_first"), ("k_split_seg", "scatter_keys"), ("k_split<sa::SrcBucketKeys", "scatter_keys"),
         ("k_bucket_hist", "pack"), ("k_bucket_starts", "bucket_starts"),
         ("k_init_rank", "init"), ("k_hist<sa::SrcRank>", "hist_rank"), ("k_hist<sa::SrcText>", "hist_text"),
         ("k_hist<sa::SrcU", "hist_u"), ("k_hist<sa::SrcKeys>", "hist_keys"),
         ("k_scan_rows", "scan"), ("k_scatter<sa::SrcRank>", "scatter_rank"),
         ("k_scatter<sa::SrcText>", "scatter_text"), ("k_scatter<sa::SrcU", "scatter_u"),
         ("k_scatter<sa::SrcKeysIota>", "scatter_iota"), ("k_pack_text", "pack"),
         ("k_scatter<sa::SrcKeys>", "scatter_keys_rs"),
         ("k_onesweep<sa::SrcKeysIota", "scatter_iota"), ("k_onesweep<sa::SrcKeys,", "scatter_keys"),
         ("k_onesweep<sa::SrcBucketIota", "scatter_first"), ("k_onesweep<sa::SrcBucketKeys", "scatter_keys"),
         ("k_pack_bucket", "pack"), ("k_window_starts", "windows"), ("k_window_max", "windows"),
         ("k_bucket_sort_lsd", "local_sort_lsd"), ("k_bucket_sort", "local_sort"),
         ("k_materialize", "sort_u_keys"), ("k_wscan_", "seg_write"), ("k_u_gather", "seg_write"),
         ("k_onesweep<sa::SrcU", "scatter_u"), ("k_onesweep<sa::SrcRank", "scatter_rank"),
         ("k_global_hist", "global_hist"), ("k_digit_base", "digit_base"), ("k_alphabet", "alphabet"),
         ("k_heads", "heads"), ("k_scan_heads", "heads_scan"),
         ("k_rerank", "rerank"), ("k_seg_count", "seg_count"), ("k_seg_scan", "seg_scan"),
         ("k_seg_write", "seg_write"), ("k_gen_text", "gen_text")]


def kind_of(name):
    for key, k in KINDS:
        if key in name:
            return k
    return None


def find(d, suffix):
    hits = sorted(glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True))
    return hits[-1] if hits else None


def main():
    tag, out = sys.argv[1], sys.argv[2]
    args = sys.argv[3:]
    n = 1 << 30
    kind = "dna"
    for i, a in enumerate(args):
        if a == "--n":
            n = int(args[i + 1])
        if a == "--kind":
            kind = args[i + 1]
    stats_csv = find(os.path.join(out, "trace"), "kernel_stats.csv")
    trace_csv = find(os.path.join(out, "trace"), "kernel_trace.csv")

    def grid(row):
        return int(float(row.get("Grid_Size") or row.get("Grid_Size_X") or 0))

    # per kind: all launches, and the full-size ones: those within 4x of the
    # kind's longest (the launches over all n suffixes, not the small
    # unsorted-set ones; persistent kernels have equal grids for both, so the
    # grid size cannot tell them apart)
    per = defaultdict(lambda: {"calls": 0, "total_ns": 0.0, "all": []})
    if trace_csv:
        with open(trace_csv) as f:
            for row in csv.DictReader(f):
                k = kind_of(row.get("Kernel_Name", ""))
                if k:
                    d = float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
                    per[k]["calls"] += 1
                    per[k]["total_ns"] += d
                    per[k]["all"].append(d)
    pmc = {}
    for name, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        c = find(os.path.join(out, sub), "counter_collection.csv")
        acc = defaultdict(lambda: defaultdict(list))
        if c:
            with open(c) as f:
                for row in csv.DictReader(f):
                    if row.get("Counter_Name") != name:
                        continue
                    k = kind_of(row.get("Kernel_Name", ""))
                    if k:
                        acc[k][(row.get("Dispatch_Id") or row.get("Correlation_Id") or len(acc[k]))].append(
                            float(row["Counter_Value"]) * 1024.0)   # KiB -> bytes, summed over the dispatch's rows
        big = {}
        for k, v in acc.items():
            tot = [sum(x) for x in v.values()]
            if tot:
                full = [x for x in tot if x >= 0.25 * max(tot)]
                big[k] = sum(full) / len(full)
        pmc[name] = big
    # SQ pass (collect.sh, one --pmc run of 8 SQ counters): per kind, the
    # full-size launches' average of each counter (whole chip, per dispatch)
    sq = defaultdict(dict)
    c = find(os.path.join(out, "sq"), "counter_collection.csv")
    if c:
        acc = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
        with open(c) as f:
            for row in csv.DictReader(f):
                k = kind_of(row.get("Kernel_Name", ""))
                if k:
                    d = row.get("Dispatch_Id") or row.get("Correlation_Id")
                    acc[k][row["Counter_Name"]][d] += float(row["Counter_Value"])
        for k, cv in acc.items():
            for cname, per_d in cv.items():
                vals = list(per_d.values())
                full = [x for x in vals if x >= 0.25 * max(vals)] if max(vals) > 0 else vals
                sq[k][cname] = sum(full) / len(full)
    fetch, write = pmc["FETCH_SIZE"], pmc["WRITE_SIZE"]
    # calibration: k_alphabet reads exactly n text bytes (16 B per lane)
    read_factor = None
    if fetch.get("alphabet"):
        read_factor = 1.0 * n / fetch["alphabet"]
    kernels = {}
    for k, v in per.items():
        full = [d for d in v["all"] if d >= 0.25 * max(v["all"])]
        e = {"calls": v["calls"], "avg_ms": v["total_ns"] / max(v["calls"], 1) / 1e6,
             "total_ms": v["total_ns"] / 1e6, "full_size_calls": len(full),
             "full_size_avg_ms": sum(full) / len(full) / 1e6}
        if k in fetch:
            e["fetch_bytes_raw"] = fetch[k]
        if k in write:
            e["write_bytes_raw"] = write[k]
        if k in fetch and k in write:
            rf = read_factor if read_factor else 2.0
            e["traffic_bytes_corrected"] = fetch[k] * rf + write[k]
        if sq.get(k):
            e["sq"] = dict(sorted(sq[k].items()))
            if sq[k].get("SQ_INSTS_LDS"):
                e["sq"]["conflict_cycles_per_lds_inst"] = sq[k].get("SQ_LDS_BANK_CONFLICT", 0.0) / sq[k]["SQ_INSTS_LDS"]
        kernels[k] = e
    bench = None
    bj = os.path.join(out, "bench.json")
    if os.path.exists(bj):
        with open(bj) as f:
            bench = json.loads(f.read())
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from hpc_suffix_array_amd._native import source_hash
    summary = {
        "tag": tag, "n": n, "kind": kind, "args": args,
        # the sources these counters measured (bench.py matches on it)
        "src_hash": (bench or {}).get("src_hash") or source_hash(),
        "read_calibration": {"kernel": "alphabet (full-n launch)", "known_read_bytes": n,
                             "factor": read_factor},
        "kernels": kernels,
        # per full-size launch, keyed like bench.py's kernel kinds
        "traffic_bytes_per_launch": {k: v["traffic_bytes_corrected"] for k, v in kernels.items()
                                     if v.get("traffic_bytes_corrected") is not None},
        "bench": bench,
    }
    here = os.path.dirname(os.path.abspath(__file__))
    with open(os.path.join(here, f"{tag}_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    if stats_csv:
        shutil.copy(stats_csv, os.path.join(here, f"{tag}_kernel_stats.csv"))
    print(json.dumps({k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                      for k, v in kernels.items()}, indent=1))


if __name__ == "__main__":
    main()
