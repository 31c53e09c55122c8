"""The benchmark entry points and the CLI contract (reference
scripts/benchmark_sequential.py, src/sequential/main_sequential.c)."""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))

CLI_TEXT = """Reading from file: test_data/banana.txt
Actual string length: 6

=== RESULTS ===
Valid suffix array: YES
Longest repeated substring: 'ana' (length: 3)
Total execution time: 0.001234 seconds

===STRUCTURED_RESULTS===
IMPLEMENTATION:sequential
TOTAL_TIME:0.001234
SA_TIME:0.001000
LCP_TIME:0.000234
===END_RESULTS===
"""


def test_parse_output_contract():
    import benchmark_sequential as B
    r = B.parse_output(CLI_TEXT)
    assert r["lrs_length"] == 3 and r["lrs_string"] == "ana"
    assert r["suffix_array_length"] == 6
    assert r["total_time"] == pytest.approx(0.001234)
    assert r["sa_time"] == pytest.approx(0.001) and r["lcp_time"] == pytest.approx(0.000234)


def test_csv_schema_is_the_references():
    import benchmark_sequential as B
    # reference scripts/benchmark_sequential.py:192-209, in order
    assert B.CSV_COLUMNS == ["file", "size_bytes", "size_mb", "backend", "time_seconds", "throughput_mb_s",
                             "throughput_chars_per_second", "lrs_length", "lrs_string", "suffix_array_length",
                             "execution_details", "total_time", "sa_time", "lcp_time", "success", "timestamp"]


def test_dataset_generator_matches_oracle(tmp_path, oracle):
    import generate_large_datasets as G
    t = G.splitmix_text(G.ALNUM, 100_000, 1)
    assert t == oracle.gen_text("alnum", 100_000, seed=1).tobytes()
    G.main(["--sizes", "1", "--out", str(tmp_path)])
    data = (tmp_path / "large" / "random_1MB.txt").read_bytes()
    assert oracle.sha256(np.frombuffer(data, np.uint8)).startswith("cd3b75303b322388")   # config 1 text


def test_cli_builds_and_refuses_without_gpu(sa_lib):
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools")], check=True)
    exe = os.path.join(ROOT, "bin", "main_sequential")
    r = subprocess.run([exe], capture_output=True, text=True)
    assert r.returncode == 1 and "Usage" in r.stdout
    if sa_lib.device_count() == 0:
        r = subprocess.run([exe, "banana"], capture_output=True, text=True)
        assert r.returncode == 1 and "no HIP device" in r.stderr


@pytest.mark.gpu
def test_cli_and_shim_on_gpu(gpu, oracle, tmp_path):
    import benchmark_sequential as B
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools")], check=True)
    files = []
    for name, text in (("banana.txt", b"banana"), ("mississippi.txt", b"mississippi"),
                       ("rand.txt", oracle.gen_text("alnum", 300_000, seed=3).tobytes())):
        p = tmp_path / name
        p.write_bytes(text)
        files.append(str(p))
    for f in files:
        t = np.frombuffer(open(f, "rb").read(), np.uint8)
        sa = oracle.sa_c(t)
        want = oracle.lrs_c(t, sa, oracle.lcp_c(t, sa)).decode("latin-1")
        for cli in (False, True):
            r = B.run_benchmark(f, use_cli=cli)
            assert r["success"], r["error"]
            assert r["lrs_string"] == want and r["lrs_length"] == len(want)
            assert r["suffix_array_length"] == len(t)
            assert "Valid suffix array: YES" in r["output"]
    out = tmp_path / "res.csv"
    assert B.main(["--files"] + files + ["--out", str(out)]) == 0
    import pandas as pd
    df = pd.read_csv(out)
    assert list(df.columns) == B.CSV_COLUMNS and len(df) == 3


@pytest.mark.gpu
def test_config1_random_1mb_through_the_harness(gpu, oracle, tmp_path):
    """configs[0]: scripts/benchmark_sequential.py on the generated 1 MiB
    random file (test_data/large/random_1MB.txt of generate_large_datasets.py)
    through the shim and the CLI, LRS and SA pinned by SURVEY.md 8(c)."""
    import benchmark_sequential as B
    import generate_large_datasets as G
    from hpc_suffix_array_amd import SuffixArray
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools")], check=True)
    G.main(["--sizes", "1", "--out", str(tmp_path)])
    f = str(tmp_path / "large" / "random_1MB.txt")
    for cli in (False, True):
        r = B.run_benchmark(f, use_cli=cli)
        assert r["success"], r["error"]
        assert (r["lrs_string"], r["lrs_length"]) == ("E31tuV", 6)
        assert r["suffix_array_length"] == 1 << 20 and "Valid suffix array: YES" in r["output"]
    out = tmp_path / "res.csv"
    assert B.main(["--files", f, "--out", str(out)]) == 0
    with SuffixArray(open(f, "rb").read()) as s:   # the drop-in symbols the shim calls
        s.build()
        assert oracle.sha256(s.sa.astype(np.int32)) == \
            "327c4c99ad49e1ae66133ef0558e0ef6b91174715ba6c02dc5f50deeec63fa56"


def test_bench_picks_the_profile_of_the_current_sources(tmp_path):
    """bench.py's roofline.traffic comes from the rocprof summary of this
    workload stamped with the current sources' hash; tags order by round and
    version (r02_bb after r02_o, r01_v30 after r01_v9), never lexically."""
    import json
    sys.path.insert(0, ROOT)
    import bench
    assert bench.tag_order("r02_bb") > bench.tag_order("r02_o") > bench.tag_order("r02_a")
    assert bench.tag_order("r01_v30") > bench.tag_order("r01_v9")
    assert bench.tag_order("r03_a") > bench.tag_order("r02_bb")

    def put(tag, **kw):
        s = dict(tag=tag, n=1 << 30, kind="dna", args=[], traffic_bytes_per_launch={"local_sort": 1.0})
        s.update(kw)
        (tmp_path / f"{tag}_summary.json").write_text(json.dumps(s))
    put("r02_o", src_hash="old")
    put("r02_bb", src_hash="head")
    put("r02_bc", src_hash="old2")
    put("r02_bd", src_hash="head", args=["--round1", "lsd"])   # another configuration: never used
    put("r02_be", src_hash="head", n=1 << 26)
    s = bench.pmc_summary(1 << 30, "dna", "head", str(tmp_path))
    assert s["tag"] == "r02_bb" and not s["stale"]
    s = bench.pmc_summary(1 << 30, "dna", "new", str(tmp_path))
    assert s["tag"] == "r02_bc" and s["stale"]
    assert bench.pmc_summary(1 << 30, "dna", "head", str(tmp_path)) is not None
    assert bench.pmc_summary(1 << 29, "dna", "head", str(tmp_path)) is None
    # the committed profiles: the latest default-workload summary is picked
    s = bench.pmc_summary(1 << 30, "dna", bench.SRC_HASH)
    assert s is not None and s["tag"] != "r02_o"


def test_reference_schedule_round_model():
    """bench.py's per-round roofline of the reference schedule follows
    SURVEY.md 8(d): P_j from D_{j-1} with D_0 = 256, B_j = n (3 rb + 2 S
    (P_j + 1)); configs[2] (1 GiB DNA) gives P = [3, 2, 3, 5, 8], 684 B per
    suffix over the five rounds (734 GB, the 91.8 ms floor)."""
    sys.path.insert(0, ROOT)
    import bench
    n = 1 << 30
    d = [17, 259, 65543, 950039036, n]
    rows = bench.model_rounds(n, d, [10.0] * 5)
    assert [r["P_model"] for r in rows] == [3, 2, 3, 5, 8]
    assert sum(r["model_bytes"] for r in rows) == 684 * n
    assert abs(sum(r["model_bytes"] for r in rows) / 8.0e12 * 1e3 - 91.8) < 0.1
    assert abs(rows[0]["frac"] - 108 * n / 10e-3 / 8.0e12) < 1e-3
    # configs[1] (64 MiB DNA): P = [3, 2, 3, 5, 7], 660 B per suffix
    m = 1 << 26
    rows = bench.model_rounds(m, [17, 259, 65543, 16744000 * 4, m], [1.0] * 5)
    assert [r["P_model"] for r in rows] == [3, 2, 3, 5, 7]
    assert sum(r["model_bytes"] for r in rows) == 660 * m


def test_scaling_harness_columns_and_commands():
    """scripts/benchmark_scaling.py: the mpi_results.csv columns of the
    reference's sweep (benchmark_mpi.py:180-210) from bench.py JSON lines, and
    the torch.distributed.run launch of N > 1 on 127.0.0.1."""
    import benchmark_scaling as S

    class A:
        steps, warmup, n, kind, no_cpu_baseline = 3, 1, 4096, "dna", False
    one = S.command(1, A, 29500)
    two = S.command(2, A, 29501)
    assert one[1].endswith("bench.py") and "--no-cpu-baseline" not in one
    assert "torch.distributed.run" in two and "--master-addr" in two and "127.0.0.1" in two
    assert "--no-cpu-baseline" in two and two[two.index("--gpus") + 1] == "2"
    res = [(1, {"ms_per_step": 40.0, "value": 2.5e10, "cpu_baseline": {"value": 1e7}}),
           (2, {"ms_per_step": 25.0, "value": 4.0e10})]
    rows = S.rows_from(res, "dna_1073741824", 1 << 30)
    assert [r["backend"] for r in rows] == ["hip_1", "hip_2"]
    assert set(S.COLUMNS) == set(rows[0])
    assert rows[1]["speedup"] == pytest.approx(1.6) and rows[1]["efficiency"] == pytest.approx(0.8)
    assert rows[0]["speedup_vs_cpu"] == pytest.approx(2500.0)
    assert S.last_json('noise\n{"a": 1}\n') == {"a": 1}
    # only verified strong-scaling lines (one string over all GPUs) enter
    assert S.rejected({"verified": True, "scaling": "strong"}) is None
    assert "scaling" in S.rejected({"verified": True, "scaling": "weak"})
    assert "verified" in S.rejected({"verified": False, "scaling": "strong"})
    assert "verified" in S.rejected({"scaling": "strong"})
