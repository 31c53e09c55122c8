"""GPU parity of the LCP array and the longest repeated substring
(sa_lcp / sa_lcp_device, replacing build_lcp_array, manber_myers.c:135-157,
and find_longest_repeated_substring, :159-182).

Bit-exact against the reference's own outputs (tests/golden), the C Kasai
restatement (oracle_lcp) on seeded inputs, the reference-recorded LRS known
answers (1 MiB, 2^30 - 1), and the analytic LCP of one repeated symbol
(LCP[r] = r) at sizes where one repeat spans the whole text -- the case the
cooperative comparison rounds exist for.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_golden_lcp(gpu, golden):
    from hpc_suffix_array_amd import lcp_array
    for name, c in golden["cases"].items():
        lcp, (ln, pos) = lcp_array(c["text"], c["sa"])
        assert lcp.dtype == np.uint32
        assert (lcp == c["lcp"]).all(), name
        t = bytes(c["text"])
        if 0 not in t:
            assert t[pos:pos + ln].hex() == c["lrs"], name


@pytest.mark.parametrize("kind", ["dna", "alnum", "ascii127", "byte256", "binary"])
@pytest.mark.parametrize("n", [1, 2, 3, 7, 8, 9, 4095, 65537, 1_000_003])
def test_lcp_vs_oracle(gpu, oracle, kind, n):
    from hpc_suffix_array_amd import lcp_array
    t = oracle.gen_text(kind, n, seed=3 * n + len(kind))
    sa = oracle.sa_c(t)
    ref = oracle.lcp_c(t, sa)
    lcp, (ln, pos) = lcp_array(t, sa)
    assert (lcp == ref).all()
    assert bytes(t[pos:pos + ln]) == oracle.lrs_c(t, sa, ref)
    w, _ = lcp_array(t, sa.astype(np.int64), width=8)
    assert w.dtype == np.int64 and (w == ref).all()


@pytest.mark.parametrize("n", [2, 9, 130, 4097, 1 << 20, (1 << 24) + 5])
def test_lcp_one_symbol(gpu, n):
    """SA = n-1 .. 0, LCP[r] = r: a single irreducible pair of length n-1."""
    from hpc_suffix_array_amd import lcp_array
    t = np.full(n, ord("a"), np.uint8)
    sa = np.arange(n - 1, -1, -1, dtype=np.uint32)
    lcp, (ln, pos) = lcp_array(t, sa)
    assert (lcp == np.arange(n, dtype=np.uint32)).all()
    assert (ln, pos) == (n - 1, 0)


def test_lcp_long_repeats(gpu, oracle):
    """Repeats of every length around the direct / cooperative boundaries
    (128 bytes, 512, 2048, ...): a random block copied at several offsets,
    periodic texts, and an unaligned text start."""
    from hpc_suffix_array_amd import lcp_array
    rng = np.random.default_rng(7)
    cases = []
    for L in (120, 127, 128, 129, 136, 511, 512, 513, 2047, 2049, 70_000):
        blk = rng.integers(97, 101, size=L, dtype=np.uint8)
        filler = rng.integers(97, 101, size=3 * L + 11, dtype=np.uint8)
        cases.append(np.concatenate([filler[:L // 2 + 3], blk, filler[L // 2 + 3:], blk, filler[:5], blk]))
    cases.append(np.tile(np.frombuffer(b"abaababa", np.uint8), 40_000))
    cases.append(np.tile(oracle.gen_text("dna", 3001, seed=2), 200))
    big = oracle.gen_text("alnum", 300_001, seed=9)
    cases.append(big[1:])                        # odd start address of the text buffer copy
    for t in cases:
        t = np.ascontiguousarray(t)
        sa = oracle.sa_c(t)
        ref = oracle.lcp_c(t, sa)
        lcp, (ln, pos) = lcp_array(t, sa)
        assert (lcp == ref).all(), len(t)
        assert bytes(t[pos:pos + ln]) == oracle.lrs_c(t, sa, ref)


def test_lcp_with_nul_bytes(gpu, oracle):
    """Bytes are compared raw (a NUL is an ordinary smallest symbol)."""
    from hpc_suffix_array_amd import lcp_array
    t = oracle.gen_text("byte256", 200_000, seed=4)
    t[::97] = 0
    sa = oracle.sa_c(t)
    lcp, _ = lcp_array(t, sa)
    assert (lcp == oracle.lcp_c(t, sa)).all()


def test_lcp_known_answers_1mib(gpu, oracle, golden):
    from hpc_suffix_array_amd import build_suffix_array, lcp_array
    for key in ("alnum_1MiB", "ascii127_1MiB", "dna_1MiB"):
        k = golden["known"][key]
        t = oracle.gen_text(k["kind"], k["n"], seed=k["seed"])
        sa = build_suffix_array(t)
        _, (ln, pos) = lcp_array(t, sa)
        assert bytes(t[pos:pos + ln]).decode() == k["lrs"], key


def test_lcp_rejects_invalid_sa(gpu, oracle):
    from hpc_suffix_array_amd import SAError, lcp_array
    t = oracle.gen_text("dna", 10_000, seed=1)
    sa = oracle.sa_c(t)
    bad = sa.copy()
    bad[3] = bad[4]
    with pytest.raises(SAError):
        lcp_array(t, bad)


def test_lcp_device_builder(gpu, oracle):
    import torch
    from hpc_suffix_array_amd import DeviceBuilder
    n = 2_000_003
    t = oracle.gen_text("dna", n, seed=6)
    d_text = torch.from_numpy(t).cuda()
    d_sa = torch.empty(n, dtype=torch.int32, device="cuda")
    d_lcp = torch.empty(n, dtype=torch.int32, device="cuda")
    b = DeviceBuilder(n)
    b.build(d_text, n, d_sa)
    ln, pos = b.lcp(d_text, n, d_sa, d_lcp, stream=torch.cuda.current_stream().cuda_stream)
    sa = d_sa.cpu().numpy().view(np.uint32)
    ref = oracle.lcp_c(t, sa)
    assert (d_lcp.cpu().numpy().view(np.uint32) == ref).all()
    assert bytes(t[pos:pos + ln]) == oracle.lrs_c(t, sa, ref)
    b.close()


@pytest.mark.slow
def test_lcp_config3_lrs_known_answer(gpu, oracle, golden):
    """configs[2] (2^30 - 1 DNA): the reference's recorded LRS."""
    import torch
    from hpc_suffix_array_amd import DeviceBuilder
    k = golden["known"]["dna_1GiB_minus_1"]
    n = k["n"]
    d_text = torch.from_numpy(oracle.gen_text("dna", n, seed=1)).cuda()
    d_sa = torch.empty(n, dtype=torch.int32, device="cuda")
    d_lcp = torch.empty(n, dtype=torch.int32, device="cuda")
    b = DeviceBuilder(n)
    b.build(d_text, n, d_sa)
    ln, pos = b.lcp(d_text, n, d_sa, d_lcp)
    assert bytes(d_text[pos:pos + ln].cpu().numpy()).decode() == k["lrs"]
    b.close()
