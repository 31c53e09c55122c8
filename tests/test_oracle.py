"""CPU tests of the oracle (test infrastructure) against the reference's
golden vectors (tests/golden, generated from the reference compiled from its
own sources) and the SHA-256 known answers of SURVEY.md 8(c)."""
import numpy as np
import pytest


def test_generator_numpy_matches_c(oracle):
    for kind in ("dna", "alnum", "ascii127", "byte256", "binary"):
        for n in (1, 2, 1000, 65537):
            assert (oracle.gen_text(kind, n, seed=3) == oracle.gen_text_c(kind, n, seed=3)).all()


def test_golden_cases(oracle, golden):
    for name, c in golden["cases"].items():
        t, sa = c["text"], c["sa"]
        got = oracle.sa_c(t)
        assert (got == sa).all(), name
        assert (oracle.sa_numpy(t) == sa).all(), name
        assert oracle.check_c(t, sa), name
        lcp = oracle.lcp_c(t, sa)
        assert (lcp == c["lcp"]).all(), name
        assert oracle.lrs_c(t, sa, lcp).hex() == c["lrs"], name


def test_reference_smoke_answers(oracle, golden):
    # Makefile:131-138 expectations of the reference
    exp = {"banana": (b"ana", [5, 3, 1, 0, 4, 2]), "mississippi": (b"issi", [10, 7, 4, 1, 0, 9, 8, 6, 3, 5, 2]),
           "abcabcabc": (b"abcabc", [6, 3, 0, 7, 4, 1, 8, 5, 2])}
    for name, (lrs, sa) in exp.items():
        c = golden["cases"][name]
        assert list(c["sa"]) == sa
        assert bytes.fromhex(c["lrs"]) == lrs


@pytest.mark.parametrize("key", ["alnum_1MiB", "ascii127_1MiB", "dna_1MiB", "byte256_1MiB"])
def test_known_answers_1mib(oracle, golden, key):
    k = golden["known"][key]
    t = oracle.gen_text(k["kind"], k["n"], seed=k["seed"])
    assert oracle.sha256(t) == k["text_sha256"]
    sa = oracle.sa_c(t)
    assert oracle.sha256(sa.astype(np.int32)) == k["sa_sha256_i32"]


def test_known_answer_64mib_text(oracle, golden):
    k = golden["known"]["dna_64MiB"]
    t = oracle.gen_text(k["kind"], k["n"], seed=k["seed"])
    assert oracle.sha256(t) == k["text_sha256"]


@pytest.mark.slow
def test_known_answer_64mib_sa(oracle, golden):
    k = golden["known"]["dna_64MiB"]
    t = oracle.gen_text(k["kind"], k["n"], seed=k["seed"])
    sa, rounds, _, _ = oracle.sa_c(t, stats=True)
    assert rounds == k["rounds"]
    assert oracle.sha256(sa.astype(np.int32)) == k["sa_sha256_i32"]


def test_checker_rejects_corruption(oracle):
    t = oracle.gen_text("dna", 5000, seed=9)
    sa = oracle.sa_c(t)
    assert oracle.check_c(t, sa)
    bad = sa.copy()
    bad[[10, 11]] = bad[[11, 10]]
    assert not oracle.check_c(t, bad)
    dup = sa.copy()
    dup[3] = dup[4]
    assert not oracle.check_c(t, dup)
    assert not oracle.is_valid_ref_c(t, dup)


def test_degenerate_rounds(oracle):
    # a x n: SA = n-1..0, rounds = ceil(log2 n) (D after the
    # round with offset k is k)
    for n in (2, 3, 1000, 1 << 12):
        t = np.full(n, ord("a"), np.uint8)
        sa, rounds, _, dj = oracle.sa_c(t, stats=True)
        assert (sa == np.arange(n - 1, -1, -1)).all()
        assert dj[-1] == n


def test_unsigned_semantics(oracle):
    # 0xFF must sort after 0x01 and the shorter of two equal runs first
    t = np.frombuffer(b"\xff\xff", np.uint8)
    assert list(oracle.sa_c(t)) == [1, 0]
    t = np.frombuffer(b"a\x00b\x00", np.uint8)
    assert list(oracle.sa_c(t)) == list(oracle.sa_numpy(t))


def test_oracle_under_sanitizers():
    """The C restatement built with AddressSanitizer + UBSan (host code only,
    oracle/Makefile `asan`) over the edge cases of SURVEY.md section 5: empty,
    one symbol, degenerate and periodic runs, bytes 0x00 / 0xFF, ragged
    sizes -- every SA O(n)-checked, LCP and LRS computed."""
    import os
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    subprocess.run(["make", "-s", "-C", os.path.join(root, "oracle"), "asan"], check=True)
    r = subprocess.run([os.path.join(root, "oracle", "build", "asan_check")], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "FAIL" not in r.stdout and "ERROR" not in r.stderr
