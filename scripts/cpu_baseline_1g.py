#!/usr/bin/env python3
"""The CPU restatement (oracle/mm_oracle.c, the reference's two-pass counting
sort, manber_myers.c:81-133) at the headline's size, one thread pinned to one
core, on the GPU box's host: configs[2]'s n = 2^30 - 1 DNA, checked against
its SHA-256 known answer (tests/golden/golden.json).  bench.py's cpu_baseline
times a bounded 64 MiB sample; this records the full-size figure once.
Prints a progress line every 30 s (a silent call is taken for a hang).

    python scripts/cpu_baseline_1g.py > profiles/<tag>_cpu_baseline_1g.txt
"""
import hashlib
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from oracle import oracle as O
    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
    k = meta["known_answers"]["dna_1GiB_minus_1"]
    n = k["n"]
    O.build_oracle()
    t = O.gen_text("dna", n, seed=1)
    core = min(os.sched_getaffinity(0))
    out = {}

    def run():
        os.sched_setaffinity(0, {core})   # this thread only (Linux: per-thread affinity)
        t0 = time.perf_counter()
        sa, rounds, _, _ = O.sa_c(t, stats=True)
        out["s"] = time.perf_counter() - t0
        out["rounds"] = rounds
        out["sha"] = hashlib.sha256(sa.astype("<i4").tobytes()).hexdigest()

    th = threading.Thread(target=run)
    t0 = time.perf_counter()
    th.start()
    while th.is_alive():
        th.join(30)
        print(f"... {time.perf_counter() - t0:.0f} s", flush=True)
    model = ""
    for line in open("/proc/cpuinfo"):
        if line.startswith("model name"):
            model = line.split(":", 1)[1].strip()
            break
    ok = out["sha"] == k["sa_sha256_i32"]
    print(json.dumps({"n": n, "kind": "dna", "seconds": round(out["s"], 2), "suffixes_per_s": n / out["s"],
                      "rounds": out["rounds"], "cores": 1, "core": core, "cpu": model,
                      "sa_sha256_matches_known_answer": ok}), flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
