#!/usr/bin/env python3
"""CPU-baseline calibration.

Times the repo's reference-identical restatement (oracle/mm_oracle.c, the
two-pass counting sort over 12-byte records of manber_myers.c:15-133)
against the reference itself compiled from its own source
(oracle/_ref/libmm.so, `make -C oracle ref`; survey container only) on the
same seeded texts, one thread pinned to one core, median of 3, with the
SA_TIME definition of main_sequential.c:97-109 (create + build).  Both SAs
must be identical (the inputs lie inside the reference's valid domain).

    python scripts/calibrate_cpu.py [--sizes 16,64] [--reps 3] [--out profiles/r02_cpu_calibration.json]

Test/benchmark infrastructure only: it runs the oracle and the reference,
never the product library.
"""
import argparse
import json
import os
import platform
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="16,64", help="MiB, comma separated")
    ap.add_argument("--kind", default="dna")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r02_cpu_calibration.json"))
    a = ap.parse_args(argv)
    from oracle import oracle as O
    O.build_oracle()
    ref = O.RefLib()
    core = min(os.sched_getaffinity(0))
    os.sched_setaffinity(0, {core})
    rows = []
    for mib in (int(x) for x in a.sizes.split(",")):
        n = mib << 20
        t = O.gen_text(a.kind, n, seed=1)
        tb = t.tobytes()
        tr, tp = [], []
        sa_r = sa_p = None
        for _ in range(a.reps):
            t0 = time.perf_counter()
            sa_r, _, _, _ = ref.run(tb)
            tr.append(time.perf_counter() - t0)
            t0 = time.perf_counter()
            sa_p = O.sa_c(t)
            tp.append(time.perf_counter() - t0)
        same = bool((sa_r.astype("int64") == sa_p.astype("int64")).all())
        mr, mp = statistics.median(tr), statistics.median(tp)
        rows.append({"kind": a.kind, "n": n, "reference_s": round(mr, 3), "restatement_s": round(mp, 3),
                     "ratio_restatement_over_reference": round(mp / mr, 3), "identical_sa": same,
                     "reference_times": [round(x, 3) for x in tr], "restatement_times": [round(x, 3) for x in tp]})
        print(json.dumps(rows[-1]), flush=True)
    out = {"cpu": cpu_model(), "core": core, "host_cpus": os.cpu_count(), "reps": a.reps,
           "reference": "oracle/_ref/libmm.so (manber_myers.c, gcc -O3 -std=c99)",
           "restatement": "oracle/build/liboracle.so (oracle/mm_oracle.c, gcc -O3 -std=c99)", "rows": rows}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    return 0 if all(r["identical_sa"] for r in rows) else 1


if __name__ == "__main__":
    sys.exit(main())
