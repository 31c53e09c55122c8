"""GPU parity: the HIP builder (through the C ABI) against the oracle.

Bit-exact SA equality with
  * the reference's own outputs (tests/golden, generated from the reference
    compiled from its sources) -- small cases, every alphabet, ragged sizes;
  * the C restatement of manber_myers.c (oracle/) on seeded inputs that the
    oracle finishes in seconds;
  * the SHA-256 known answer of config 2 (64 MiB DNA);
and size-independent properties (O(n) checker, analytic degenerate SA) at
larger sizes.
"""
import ctypes
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_golden_cases_ex(gpu, golden):
    from hpc_suffix_array_amd import build_suffix_array, check_suffix_array
    for name, c in golden["cases"].items():
        got = build_suffix_array(c["text"])
        assert got.dtype == np.uint32
        assert (got == c["sa"]).all(), name
        assert check_suffix_array(c["text"], got), name


def test_golden_cases_dropin(gpu, golden):
    """The six drop-in symbols, exactly as a reference caller uses them."""
    from hpc_suffix_array_amd import SuffixArray
    for name, c in golden["cases"].items():
        t = bytes(c["text"])
        if 0 in t:      # the drop-in truncates at NUL like strncpy (manber_myers.c:57)
            continue
        with SuffixArray(t) as s:
            s.build()
            assert (s.sa == c["sa"].astype(np.int32)).all(), name
            s.build_lcp()
            assert (s.lcp == c["lcp"].astype(np.int32)).all(), name
            lrs = s.longest_repeated_substring()
            assert (lrs or b"").hex() == c["lrs"], name
            assert s.is_valid(), name


def test_int64_output(gpu, oracle):
    from hpc_suffix_array_amd import build_suffix_array
    t = oracle.gen_text("alnum", 100_003, seed=5)
    got = build_suffix_array(t, width=8)
    assert got.dtype == np.int64
    assert (got == oracle.sa_c(t).astype(np.int64)).all()


@pytest.mark.parametrize("schedule", ["packed", "reference"])
@pytest.mark.parametrize("kind", ["dna", "alnum", "ascii127", "byte256", "binary"])
@pytest.mark.parametrize("n", [1, 2, 3, 4095, 4096, 4097, 65535, 1 << 17, 1_000_003, 4_194_305])
def test_random_vs_oracle(gpu, oracle, kind, n, schedule):
    from hpc_suffix_array_amd import build_suffix_array
    t = oracle.gen_text(kind, n, seed=n + len(kind))
    got, st = build_suffix_array(t, return_stats=True, schedule=schedule)
    ref, rounds, _, dj = oracle.sa_c(t, stats=True)
    assert (got == ref).all()
    if n > 1 and schedule == "reference":
        # the reference schedule reproduces manber_myers.c round for round
        assert st["rounds"] == rounds
        assert st["distinct"] == dj
    if n > 1:
        assert st["distinct"][-1] == n


@pytest.mark.parametrize("kind", ["dna", "alnum", "byte256", "binary"])
def test_reference_rerank_permutation(gpu, oracle, kind):
    """The reference schedule's re-rank as a partition by index
    (sa_permute.h) forced at every size: one level (n <= 2^22), two levels
    with 2 / 4 sub-bins, ragged last bins and sub-bins; D_j stay the
    reference's round for round."""
    from hpc_suffix_array_amd import build_suffix_array
    for n in (2, 3, 4095, 16385, 100_003, (1 << 22) + 1, 3 * (1 << 21) + 7):
        t = oracle.gen_text(kind, n, seed=n + 3)
        got, st = build_suffix_array(t, return_stats=True, schedule="reference", debug=("perm_always",))
        ref, rounds, _, dj = oracle.sa_c(t, stats=True)
        assert (got == ref).all(), (kind, n)
        assert st["rounds"] == rounds and st["distinct"] == dj, (kind, n)
    t = np.full(70_001, ord("a"), np.uint8)
    got = build_suffix_array(t, schedule="reference", debug=("perm_always",))
    assert (got == np.arange(70_000, -1, -1, dtype=np.uint32)).all()


@pytest.mark.parametrize("debug", [(), ("no_xq",)])
def test_reference_lsd_queues(gpu, oracle, debug):
    """The reference schedule's LSD passes with per-XCD queues of tiles
    (sa_lsd.h XQ: stable in (digit, tile) order, per-queue look-backs and
    next-pass counts; packed and unpacked 12-byte passes) and without
    (debug no_xq): SA, round count and every D_j equal the oracle's."""
    from hpc_suffix_array_amd import build_suffix_array
    for kind, n in (("dna", 3_000_017), ("byte256", 1 << 21), ("alnum", 1_500_007), ("binary", 600_001)):
        t = oracle.gen_text(kind, n, seed=n + 11)
        got, st = build_suffix_array(t, return_stats=True, schedule="reference", debug=debug)
        ref, rounds, _, dj = oracle.sa_c(t, stats=True)
        assert (got == ref).all(), (kind, n, debug)
        assert st["rounds"] == rounds and st["distinct"] == dj, (kind, n, debug)


@pytest.mark.parametrize("kind", ["dna", "alnum", "ascii127", "byte256"])
def test_key1_round_two(gpu, oracle, kind):
    """The first round after a sparse bucketed round 1 sorts its members by
    key1(x + K) rebuilt from the text (SrcUKey1), which orders and ties them
    as rank[x + K] does; debug "no_key1_round" takes the ranks by the sample
    search instead.  Same SA, same D_j, as the oracle."""
    from hpc_suffix_array_amd import build_suffix_array
    n = 2_500_001
    t = oracle.gen_text(kind, n, seed=17)
    t[-40:] = t[:40]   # a repeat at the end: short suffixes in later rounds
    ref = oracle.sa_c(t)
    got, st = build_suffix_array(t, return_stats=True)
    alt, st_alt = build_suffix_array(t, return_stats=True, debug=("no_key1_round",))
    assert st["round1"] == "bucketed" and st["sparse_ranks"], st
    assert (got == ref).all() and (alt == ref).all()
    assert st["distinct"] == st_alt["distinct"]
    # round 1 leaves the key1 samples out unless a later round searches
    # them (k_key1_samples): many planted repeats keep members after round 2,
    # whose x + h land all over the text (mostly outside the set)
    rng = np.random.default_rng(29)
    u = oracle.gen_text(kind, n, seed=31)
    src = rng.integers(0, n - 200, 300)
    dst = rng.integers(0, n - 200, 300)
    for a, b, ln in zip(src, dst, rng.integers(40, 160, 300)):
        u[b:b + ln] = u[a:a + ln].copy()
    ref = oracle.sa_c(u)
    got, st = build_suffix_array(u, return_stats=True)
    alt, st_alt = build_suffix_array(u, return_stats=True, debug=("no_key1_round",))
    assert st["sparse_ranks"] and st["rounds"] > 2, st
    assert (got == ref).all() and (alt == ref).all()
    assert st["distinct"] == st_alt["distinct"]


def test_alphabet_late_values(gpu, oracle):
    """The alphabet pass stops a wave once its lanes have seen all 256 byte
    values (k_alphabet): texts where some values appear only near the end,
    or only once, still report every value present -- sigma and the SA
    agree with the oracle; byte256 text takes the 8-byte window first pass."""
    from hpc_suffix_array_amd import build_suffix_array
    rng = np.random.default_rng(13)
    n = 3_000_017
    # all 256 values early (waves stop), and a text missing 0x7F but at its end
    t = rng.integers(0, 256, n, dtype=np.uint8)
    t[t == 0x7F] = 0x80
    t[-1] = 0x7F
    cases = [t]
    # every value once, each in a different part of a mostly-'a' text
    u = np.full(n, ord("a"), np.uint8)
    u[rng.choice(n, 256, replace=False)] = np.arange(256, dtype=np.uint8)
    cases.append(u)
    # random bytes without one value at all (255 present)
    v = rng.integers(0, 255, n, dtype=np.uint8)
    cases.append(v)
    for x, sigma in zip(cases, (256, 256, 255)):
        got, st = build_suffix_array(x, return_stats=True)
        assert st["sigma"] == sigma, (st["sigma"], sigma)
        assert (got == oracle.sa_c(x)).all()


@pytest.mark.parametrize("schedule", ["packed", "reference"])
@pytest.mark.parametrize("radix", ["onesweep", "reduce_scan"])
def test_radix_algorithms(gpu, oracle, schedule, radix):
    """Both radix sorts (single-pass look-back / reduce-then-scan) under both
    schedules, across tile and chunk boundaries."""
    from hpc_suffix_array_amd import build_suffix_array
    for kind, n in (("dna", 4096 * 3 + 17), ("byte256", 1 << 18), ("alnum", 2_500_001), ("binary", 333_333)):
        t = oracle.gen_text(kind, n, seed=n)
        got = build_suffix_array(t, schedule=schedule, radix=radix)
        assert (got == oracle.sa_c(t)).all(), (kind, n)


@pytest.mark.parametrize("init_chars", [1, 2, 3, 5])
@pytest.mark.parametrize("kind", ["dna", "binary", "alnum"])
def test_packed_short_first_key(gpu, oracle, kind, init_chars):
    """A short first key leaves most suffixes unsorted: exercises the
    unsorted-set doubling rounds (compaction, (g, rank[i+h]) keys, SA/rank
    updates through the position map)."""
    from hpc_suffix_array_amd import build_suffix_array
    for n in (5, 777, 70_001, 1_000_000):
        t = oracle.gen_text(kind, n, seed=init_chars * 7 + n)
        got, st = build_suffix_array(t, return_stats=True, init_chars=init_chars)
        assert st["init_chars"] == init_chars
        assert (got == oracle.sa_c(t)).all(), (kind, n, init_chars)
        assert st["distinct"][-1] == n


def test_known_answers_1mib(gpu, oracle, golden):
    from hpc_suffix_array_amd import build_suffix_array
    for key in ("alnum_1MiB", "ascii127_1MiB", "dna_1MiB", "byte256_1MiB"):
        k = golden["known"][key]
        t = oracle.gen_text(k["kind"], k["n"], seed=k["seed"])
        got = build_suffix_array(t)
        assert oracle.sha256(got.astype(np.int32)) == k["sa_sha256_i32"], key


@pytest.mark.parametrize("schedule", ["packed", "reference"])
def test_config2_64mib_dna_known_answer(gpu, oracle, golden, schedule):
    """configs[1]: 64 MiB random DNA on 1 MI355X, bit-exact vs sequential."""
    from hpc_suffix_array_amd import build_suffix_array
    k = golden["known"]["dna_64MiB"]
    t = oracle.gen_text("dna", k["n"], seed=k["seed"])
    assert oracle.sha256(t) == k["text_sha256"]
    got, st = build_suffix_array(t, return_stats=True, schedule=schedule)
    if schedule == "reference":
        assert st["rounds"] == k["rounds"]
    assert oracle.sha256(got.astype(np.int32)) == k["sa_sha256_i32"]


@pytest.mark.parametrize("schedule", ["packed", "reference"])
@pytest.mark.parametrize("n", [2, 17, 4096, 65537, 1 << 20, (1 << 22) + 3])
def test_degenerate(gpu, n, schedule):
    """configs[4] shape: one repeated symbol, log2 n rounds, analytic SA
    (packed: the tied-block pivot rounds, and the split ones for comparison)."""
    from hpc_suffix_array_amd import build_suffix_array
    for dbg in ((), ("no_tied",)) if schedule == "packed" else ((),):
        got, st = build_suffix_array(np.full(n, ord("a"), np.uint8), return_stats=True, schedule=schedule, debug=dbg)
        assert (got == np.arange(n - 1, -1, -1, dtype=np.uint32)).all(), dbg
        assert st["distinct"][-1] == n


@pytest.mark.parametrize("mode", ["tied", "split", "no_pivot"])
def test_pivot_split_rounds(gpu, oracle, mode):
    """Unsorted-set rounds with large groups by the three-way pivot split
    (sa_pivot.h): periodic texts with sparse noise (a dominant key per group,
    plus members below and above the pivot), runs of one symbol inside random
    text, and a short first key on random DNA (many distinct keys per group:
    the split gives up and the full sort runs).  "tied" (default): tied blocks
    straight to the next unsorted set; "split": debug "no_tied"
    (SA_DEBUG_NO_TIED), tied blocks through the sorted output and segments();
    "no_pivot" (SA_DEBUG_NO_PIVOT): the full LSD sort."""
    from hpc_suffix_array_amd import build_suffix_array
    dbg = {"tied": (), "split": ("no_tied",), "no_pivot": ("no_pivot",)}[mode]
    rng = np.random.default_rng(7)
    cases = []
    for period, noise, n in ((b"ab", 0.002, 400_003), (b"abc", 0.01, 300_001), (b"aab", 0.0005, 1 << 20)):
        t = np.frombuffer((period * (n // len(period) + 1))[:n], np.uint8).copy()
        hit = rng.random(n) < noise
        t[hit] = rng.integers(ord("a"), ord("e"), int(hit.sum()), dtype=np.uint8)
        cases.append(t)
    t = oracle.gen_text("dna", 500_000, seed=3)
    t[100_000:260_000] = ord("G")
    cases.append(t)
    # runs of one symbol with random lengths: many groups per round, tied
    # blocks of one member (sorted at once) and of many
    lens = rng.integers(1, 600, 3000)
    t = np.repeat(rng.integers(ord("a"), ord("d"), len(lens), dtype=np.uint8), lens)
    cases.append(t)
    for t in cases:
        got = build_suffix_array(t, debug=dbg)
        assert (got == oracle.sa_c(t)).all(), (len(t), mode)
    for n in (70_001, 1_000_000):
        t = oracle.gen_text("dna", n, seed=n)
        got = build_suffix_array(t, init_chars=2, debug=dbg)
        assert (got == oracle.sa_c(t)).all(), (n, mode)


@pytest.mark.parametrize("schedule", ["packed", "reference"])
def test_periodic(gpu, oracle, schedule):
    from hpc_suffix_array_amd import build_suffix_array
    base = oracle.gen_text("alnum", 1000, seed=11)
    t = np.tile(base, 300)
    assert (build_suffix_array(t, schedule=schedule) == oracle.sa_c(t)).all()
    # short period, long repeats: most suffixes stay unsorted for many rounds
    t = np.tile(np.frombuffer(b"abaababa", np.uint8), 40_000)
    assert (build_suffix_array(t, schedule=schedule) == oracle.sa_c(t)).all()


def test_checker_detects_corruption(gpu, oracle):
    from hpc_suffix_array_amd import check_suffix_array
    t = oracle.gen_text("dna", 300_000, seed=2)
    sa = oracle.sa_c(t)
    assert check_suffix_array(t, sa)
    bad = sa.copy()
    bad[[1000, 1001]] = bad[[1001, 1000]]
    assert not check_suffix_array(t, bad)
    dup = sa.copy()
    dup[7] = dup[8]
    assert not check_suffix_array(t, dup)
    oob = sa.copy()
    oob[0] = len(t)
    assert not check_suffix_array(t, oob)


@pytest.mark.parametrize("n", [1, 2, 3, 100, 8191, 8192, 8193, 16383, 16384, 16385, 1 << 21, (1 << 22) + 5,
                               5_000_011])
def test_checker_permutation_passes(gpu, oracle, n):
    """The permutation checker (sa_check.h) at sizes around its sub-bins
    (2^13 / 2^14) and bins (one level up to 2^21 / 2^22, two above), against
    corruptions placed inside a sub-bin, across a sub-bin boundary, at both
    ends, and whole-array permutations that keep SA a permutation."""
    from hpc_suffix_array_amd import check_suffix_array
    rng = np.random.default_rng(n)
    t = oracle.gen_text("dna" if n > 3 else "alnum", n, seed=n)
    sa = oracle.sa_c(t)
    assert check_suffix_array(t, sa)
    if n == 1:
        assert not check_suffix_array(t, np.array([1], np.uint32))
        return
    cases = {"swap_first": (0, 1), "swap_last": (n - 2, n - 1)}
    for k in (8191, 8192, 16383, 16384):   # sub-bin boundaries of pass B / pass A
        if k < n:
            cases[f"swap_{k}"] = (k - 1, k)
    for name, (i, j) in cases.items():
        bad = sa.copy()
        bad[[i, j]] = bad[[j, i]]
        assert not check_suffix_array(t, bad), name
    dup = sa.copy()
    dup[rng.integers(0, n)] = dup[rng.integers(0, n)] if n > 2 else dup[0]
    if not (dup == sa).all():
        assert not check_suffix_array(t, dup)
    oob = sa.copy()
    oob[rng.integers(0, n)] = n + int(rng.integers(0, 1000))
    assert not check_suffix_array(t, oob)
    assert not check_suffix_array(t, sa[::-1].copy())
    assert not check_suffix_array(t, np.arange(n, dtype=np.uint32)) or (sa == np.arange(n)).all()
    if n > 64:
        sh = sa.copy()
        k = int(rng.integers(0, n - 32))
        sh[k:k + 32] = rng.permutation(sh[k:k + 32])
        assert check_suffix_array(t, sh) == (sh == sa).all()


def test_device_builder_torch(gpu, oracle):
    """Device-resident path (what bench.py times), torch buffers in HBM."""
    import torch
    from hpc_suffix_array_amd import DeviceBuilder
    n = 3_000_017
    t = oracle.gen_text("dna", n, seed=4)
    d_text = torch.from_numpy(t).cuda()
    d_sa = torch.empty(n, dtype=torch.int32, device="cuda")
    b = DeviceBuilder(n)
    st = b.build(d_text, n, d_sa, stream=torch.cuda.current_stream().cuda_stream, profile=True)
    torch.cuda.synchronize()
    got = d_sa.cpu().numpy().view(np.uint32)
    assert (got == oracle.sa_c(t)).all()
    assert b.check(d_text, n, d_sa)
    assert st["kernels"]["scatter_keys"]["launches"] > 0
    assert abs(sum(st["round_ms"]) - st["total_ms"]) < 0.5 * st["total_ms"] + 5
    b.close()


@pytest.mark.slow
def test_config3_1gib_minus_1_known_answer(gpu, oracle, golden):
    """configs[2] at the largest n the reference handles (2^30 - 1)."""
    import torch
    from hpc_suffix_array_amd import DeviceBuilder
    k = golden["known"]["dna_1GiB_minus_1"]
    n = k["n"]
    t = oracle.gen_text("dna", n, seed=1)
    d_text = torch.from_numpy(t).cuda()
    del t
    d_sa = torch.empty(n, dtype=torch.int32, device="cuda")
    b = DeviceBuilder(n)
    st = b.build(d_text, n, d_sa)
    # the packed schedule (default) takes fewer, longer rounds than the
    # reference's 5 (the h-prefix lengths per round are checked elsewhere)
    assert st["schedule"] == "packed" and st["rounds"] <= k["rounds"]
    assert b.check(d_text, n, d_sa)
    sa = d_sa.cpu().numpy()
    assert oracle.sha256(sa) == k["sa_sha256_i32"]
    b.close()


@pytest.mark.slow
def test_config5_degenerate_1gib(gpu):
    """configs[4]: 1 GiB degenerate input ('a' x 2^30) on one MI355X.  The SA
    is analytic (n-1, ..., 0); the packed schedule takes 26 rounds (first key
    63 symbols, then h = 63 * 2^j up to 2^31 > 2^30: prefix lengths beyond
    2^31 are handled in 64 bits; the reference needs 30 rounds,
    manber_myers.c:97, and cannot run n = 2^30 at all)."""
    import hashlib

    import torch
    from hpc_suffix_array_amd import DeviceBuilder
    n = 1 << 30
    d_text = torch.full((n,), ord("a"), dtype=torch.uint8, device="cuda")
    d_sa = torch.empty(n, dtype=torch.int32, device="cuda")
    b = DeviceBuilder(n)
    st = b.build(d_text, n, d_sa)
    assert st["rounds"] == 26, st["rounds"]
    assert st["prefix_len"][-1] == 63 << 25 and st["distinct"][-1] == n
    assert st["distinct"][:3] == [63, 126, 252]
    want = torch.arange(n - 1, -1, -1, dtype=torch.int32, device="cuda")
    assert torch.equal(d_sa, want)
    del want
    assert b.check(d_text, n, d_sa)
    # the same answer as a hash of the host copy (numpy's reversed arange)
    got = hashlib.sha256(d_sa.cpu().numpy().tobytes()).hexdigest()
    assert got == hashlib.sha256(np.arange(n - 1, -1, -1, dtype=np.int32).tobytes()).hexdigest()
    b.close()


def _single_rank_group():
    import socket

    import torch
    import torch.distributed as dist
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))


def test_distributed_hip_single_rank(gpu, oracle):
    """The multi-GPU drivers with the HIP local phases and RCCL collectives at
    world size 1 (the box has one GPU; world sizes 2-3 run under gloo in
    tests/test_distributed.py): the range-partitioned build (sa_dist_*) on
    every alphabet, ragged sizes, periodic text (several request rounds), and
    its sample-sort fallback (one repeated symbol)."""
    import torch
    import torch.distributed as dist
    from hpc_suffix_array_amd.distributed import DistributedSA, HipOps, HipRangeOps, SampleSortSA, gather_sa
    _single_rank_group()
    try:
        ops = HipRangeOps(1 << 22, 0)
        cases = [("dna", oracle.gen_text("dna", 3_000_017, seed=8), "range"),
                 ("alnum", oracle.gen_text("alnum", 1_500_007, seed=9), "range"),
                 ("byte256", oracle.gen_text("byte256", 2_000_003, seed=2), "range"),
                 ("ascii127", oracle.gen_text("ascii127", 65_537, seed=3), "range"),
                 ("binary", oracle.gen_text("binary", 1_000_003, seed=4), "range"),
                 # too short for the bucket layout (K <= s): the sample-sort path
                 ("tiny", np.frombuffer(b"banana", np.uint8), "sample-sort"),
                 ("periodic", np.tile(oracle.gen_text("alnum", 1000, seed=11), 300), "range"),
                 ("degenerate", np.full(70_000, ord("a"), np.uint8), "sample-sort")]
        for name, t, path in cases:
            text = torch.from_numpy(t.copy()).cuda()
            d = DistributedSA(ops)
            sa_local, sa_off = d.build(text, len(t))
            assert d.stats["path"] == path, (name, d.stats)
            sa = gather_sa(sa_local, sa_off, len(t)).cpu().numpy()
            assert (sa == oracle.sa_c(t).astype(np.int64)).all(), name
        # the sample-sort driver on its own
        hops = HipOps(1 << 22, 0)
        for t in (oracle.gen_text("dna", 300_017, seed=8), np.tile(np.frombuffer(b"abaababa", np.uint8), 9_000)):
            text = torch.from_numpy(t.copy()).cuda()
            sa = gather_sa(SampleSortSA(hops).build(text, len(t)), 0, len(t)).cpu().numpy()
            assert (sa == oracle.sa_c(t).astype(np.int64)).all()
        # running max across tile boundaries (4096 values per tile)
        g = torch.Generator().manual_seed(5)
        for m in (1, 63, 4096, 4097, 300_001):
            v = torch.randint(-1, 1 << 40, (m,), generator=g, dtype=torch.int64)
            v[torch.rand(m, generator=g) < 0.7] = -1
            got = hops.running_max(v.cuda()).cpu()
            assert torch.equal(got, torch.cummax(v, 0)[0]), m
        # the sample-sort driver's scan / search / compaction kernels against torch
        for m in (1, 63, 4096, 4097, 300_001):
            mask = torch.rand(m, generator=g) < 0.3
            x = torch.randint(0, 1 << 20, (m,), generator=g, dtype=torch.int64)
            assert torch.equal(hops.select(mask.cuda()).cpu(), mask.nonzero().squeeze(1)), m
            assert hops.count_true(mask.cuda()) == int(mask.sum()), m
            assert torch.equal(hops.cumsum(mask.cuda()).cpu(), torch.cumsum(mask.to(torch.int64), 0)), m
            assert torch.equal(hops.cumsum(x.cuda()).cpu(), torch.cumsum(x, 0)), m
            xs = torch.sort(x).values
            q = torch.randint(0, (1 << 20) + 5, (5000,), generator=g, dtype=torch.int64)
            q[:3] = torch.tensor([0, int(xs[0]), int(xs[-1])])
            for right in (False, True):
                assert torch.equal(hops.count_below(xs.cuda(), q.cuda(), right=right).cpu(),
                                   torch.searchsorted(xs, q, right=right)), (m, right)
        # owner-side scatter: in-range writes land, out-of-range ones are refused
        dst = torch.full((8,), -1, dtype=torch.int64, device="cuda")
        hops.scatter(dst, torch.tensor([12, 10], dtype=torch.int64, device="cuda"), 10,
                     torch.tensor([5, 7], dtype=torch.int64, device="cuda"))
        assert dst.tolist() == [7, -1, 5, -1, -1, -1, -1, -1]
        from hpc_suffix_array_amd._native import SAError
        with pytest.raises(SAError):
            hops.scatter(dst, torch.tensor([9, 18], dtype=torch.int64, device="cuda"), 10,
                         torch.tensor([1, 2], dtype=torch.int64, device="cuda"))
        assert dst.tolist() == [7, -1, 5, -1, -1, -1, -1, -1]
        # zero-length inputs of the sample-sort building blocks (n < world size)
        e = torch.empty(0, dtype=torch.int64, device="cuda")
        assert hops.pack_keys(torch.zeros(4, dtype=torch.uint8, device="cuda"), 4, 2, 2, [0] * 256, 5, 3).numel() == 0
        assert hops.argsort(e, 8)[0].numel() == 0 and hops.gather(e, e).numel() == 0
        assert hops.running_max(e).numel() == 0
        hops.scatter(e.clone(), e, 0, e)
        eb = torch.empty(0, dtype=torch.bool, device="cuda")
        assert hops.select(eb).numel() == 0 and hops.count_true(eb) == 0 and hops.cumsum(e).numel() == 0
        assert hops.count_below(e, e).numel() == 0
    finally:
        dist.destroy_process_group()


def _multi_rank_worker(rank, world, port, q, large=False):
    """One rank of a world sharing the box's GPU: HIP phases on cuda:0, the
    collectives through a gloo group (staged via host memory).  large: one
    DNA text of 402 M suffixes generated on the GPU, the gathered SA compared
    with the single-GPU build (too large for the CPU oracle)."""
    import os
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch
    import torch.distributed as dist
    from hpc_suffix_array_amd.distributed import DistributedSA, HipRangeOps, gather_sa
    from oracle import oracle as O
    import faulthandler
    logdir = os.path.join(root, "gpurun_out")
    os.makedirs(logdir, exist_ok=True)
    log = open(os.path.join(logdir, f"multi_rank_w{world}_r{rank}.log"), "w")
    os.dup2(log.fileno(), 2)   # the library's SA_TRACE lines and faulthandler land in the log
    os.environ["SA_DIST_TRACE"] = "1"
    faulthandler.dump_traceback_later(40, exit=True, file=log)   # a hung rank names its stack

    def say(*a):
        print(*a, file=log, flush=True)

    torch.cuda.set_device(0)
    say("init")
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    say("group up")
    try:
        # the workspace reserved up front (sa_dist_reserve) for the largest case
        ops = HipRangeOps(3_000_017, 0, world=world) if not large else HipRangeOps(0, 0)
        ops.profile = True   # round 1's sa_stats: which record path ran
        res = {}
        if large:
            from hpc_suffix_array_amd import DeviceBuilder
            n = 3 * (1 << 27) + 17
            t = torch.empty(n, dtype=torch.uint8, device="cuda")
            ops.b.generate_text(t, n, b"ACGT", seed=5)
            torch.cuda.synchronize()
            say("build large")
            d = DistributedSA(ops)
            sa_local, sa_off = d.build(t, n)
            say("built large", d.stats)
            # each rank compares its slice with the same slice of the
            # single-GPU build (a 3 GiB gather through gloo would take minutes)
            b = DeviceBuilder(n, device=0)
            want = torch.empty(n, dtype=torch.int32, device="cuda")
            b.build(t, n, want)
            torch.cuda.synchronize()
            m = sa_local.numel()
            mine = sa_local.to(torch.int64) & 0xFFFFFFFF
            ref = want[int(sa_off): int(sa_off) + m].to(torch.int64) & 0xFFFFFFFF
            ok = torch.tensor([1 if bool((mine == ref).all().item()) else 0, m], dtype=torch.int64)
            b.close()
            del want
            dist.all_reduce(ok[:1], op=dist.ReduceOp.MIN)
            tot = ok[1:].clone()
            dist.all_reduce(tot)
            say("checked large", ok.tolist(), tot.tolist())
            if rank == 0:
                res["dna_large"] = (bool(ok[0] == 1 and int(tot[0]) == n), d.stats["path"], len(d.stats["unsorted"]),
                                    ops.round1_stats.to_dict()["round1_layout"])
                q.put(res)
            return
        for name, kind, n, seed in (("dna", "dna", 3_000_017, 8), ("byte256", "byte256", 2_000_003, 2),
                                    ("alnum", "alnum", 1_048_576, 1), ("binary", "binary", 1_000_003, 4),
                                    ("periodic", None, 300_000, 11), ("degenerate", None, 70_001, 0),
                                    ("dna_overflow", "dna", 2_000_003, 9), ("dna_counted", "dna", 2_000_003, 9),
                                    ("byte256_overflow", "byte256", 2_000_003, 3),
                                    ("alnum_overflow", "alnum", 1_048_576, 5)):
            # *_overflow: record stripes of half their share (the round runs
            # again with the counting scan) -- the packed DNA, the IDENT
            # (byte256) and the non-power-of-two record kernels; dna_counted:
            # the counting scan
            ops.b.set_debug(("pad_overflow",) if name.endswith("_overflow") else
                            ("no_pad",) if name == "dna_counted" else ())
            if name == "periodic":
                t = np.tile(O.gen_text("alnum", 1000, seed=seed), 300)
            elif name == "degenerate":
                t = np.full(n, ord("a"), np.uint8)
            else:
                t = O.gen_text(kind, n, seed=seed)
            say("build", name)
            d = DistributedSA(ops)
            if name in ("dna", "alnum", "periodic", "degenerate"):
                # the bench's input: this rank's slice only, gathered by the build
                from hpc_suffix_array_amd.distributed import text_chunk
                C = text_chunk(len(t), world)
                sl = torch.from_numpy(t[min(len(t), rank * C): min(len(t), (rank + 1) * C)].copy()).cuda()
                sa_local, sa_off = d.build_sliced(sl, len(t))
                if d.stats["path"] == "range":
                    R = len(d.stats["unsorted"])
                    assert d.stats["collectives"] >= 3 + R + 2 * (R - 1), d.stats
            else:
                sa_local, sa_off = d.build(torch.from_numpy(t).cuda(), len(t))
            say("built", name, d.stats)
            sa = gather_sa(sa_local, sa_off, len(t))
            say("gathered", name)
            if rank == 0:
                want = O.sa_c(t).astype(np.int64)
                res[name] = (bool((sa.cpu().numpy() == want).all()), d.stats["path"], len(d.stats["unsorted"]),
                             ops.round1_stats.to_dict()["round1_segments"])
        ops.b.set_debug(())
        if rank == 0:
            q.put(res)
    except BaseException:
        import traceback
        say(traceback.format_exc())
        q.put({"error": (rank, traceback.format_exc())})
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4, 5])
def test_distributed_hip_multi_rank(gpu, world):
    """The range-partitioned build with real HIP phases on 2-5 ranks (all on
    the box's one GPU; the 8-GPU RCCL run is the driver's): cuts into
    unequal ranges, rank requests answered by other ranks, several doubling
    rounds (periodic text), the sample-sort fallback (one symbol) -- every SA
    equal to the oracle's.  From 4 ranks a range holds <= 0.3 n suffixes and
    round 1 sorts records emitted by k_bucket_hist<.., 3> into striped
    regions (or, forced / overflowed, counted and emitted by <.., 1 / 2>;
    k_split_list) instead of filtering the text in k_split_text."""
    _multi_rank(world)


@pytest.mark.slow
def test_distributed_hip_multi_rank_large(gpu):
    """Four ranks on one GPU at n = 3 * 2^27 + 17 DNA: ~100 M suffixes per
    range, buckets large enough that each rank's local sort takes the fixed-
    span 32-bit kernel (k_bucket_sort), checked against the single-GPU build."""
    res = _multi_rank(4, large=True)
    assert res["dna_large"][0] and res["dna_large"][1] == "range", res
    # ~100 M suffixes per range: the second pass by per-XCD queues (sa_split.h SegXq)
    assert res["dna_large"][3]["xq"], res


def _multi_rank(world, large=False):
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_multi_rank_worker, args=(r, world, port, q, large)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    assert "error" not in res, res.get("error")
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if large:
        return res
    for name, (ok, path, rounds, seg) in res.items():
        assert ok, (name, world)
        assert path == ("sample-sort" if name == "degenerate" else "range"), (name, path)
    assert res["periodic"][2] >= 4, res["periodic"]
    # ranges of <= 0.3 n (world >= 4) take the records; one striped scan of
    # the text unless forced off or overflowed
    listed = world >= 4
    assert res["dna"][3] == ("striped-records" if listed else "exact"), (world, res["dna"])
    for name in ("dna_overflow", "byte256_overflow", "alnum_overflow"):
        assert res[name][3] == ("striped-records-overflow" if listed else "exact"), (world, name, res[name])
    assert res["dna_counted"][3] == "exact", (world, res["dna_counted"])


@pytest.mark.slow
def test_distributed_hip_config4_shape(gpu, oracle, golden):
    """configs[3]'s path at the largest size one box holds: the range-
    partitioned driver at world size 1 on byte256 text (NULs and bytes >=
    0x80 included) of n = 2^31 + 17 suffixes -- 32-bit index fields in the
    bucket items (ib = 32), 18-bit buckets, 64-bit prefix lengths -- checked
    by the O(n) checker; plus the byte256 1 MiB known answer through the same
    driver."""
    import torch
    import torch.distributed as dist
    from hpc_suffix_array_amd.distributed import DistributedSA, HipRangeOps, gather_sa
    _single_rank_group()
    try:
        ops = HipRangeOps(0, 0)
        k = golden["known"]["byte256_1MiB"]
        t = oracle.gen_text("byte256", k["n"], seed=k["seed"])
        d = DistributedSA(ops)
        sa_local, sa_off = d.build(torch.from_numpy(t).cuda(), len(t))
        assert d.stats["path"] == "range" and sa_off == 0
        got = gather_sa(sa_local, sa_off, len(t)).cpu().numpy().astype(np.int32)
        assert oracle.sha256(got) == k["sa_sha256_i32"]
        n = (1 << 31) + 17
        text = torch.empty(n, dtype=torch.uint8, device="cuda")
        ops.b.generate_text(text, n, bytes(range(256)), seed=1)
        d = DistributedSA(ops)
        sa_local, sa_off = d.build(text, n)
        torch.cuda.synchronize()
        assert d.stats["path"] == "range" and d.stats["m"] == n, d.stats
        assert d.stats["unsorted"][-1] == 0
        assert ops.b.check(text, n, sa_local)   # the context's buffers are free again
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["dna", "alnum", "ascii127", "byte256", "binary"])
@pytest.mark.parametrize("n", [2, 3, 17, 4097, 65537, 1_000_003, 2_500_001])
def test_bucketed_round1_vs_oracle(gpu, oracle, kind, n):
    """First round as two bucket passes + per-window LDS sort (sa_bucket.h),
    forced at every size: short texts (every suffix shorter than the bucket
    prefix), many tiny windows, and 1-2.5 M suffixes (the auto threshold)."""
    from hpc_suffix_array_amd import build_suffix_array
    t = oracle.gen_text(kind, n, seed=7 * n + len(kind))
    got, st = build_suffix_array(t, return_stats=True, round1="bucketed")
    assert (got == oracle.sa_c(t)).all()
    assert st["distinct"][-1] == n
    if n >= 65537:
        assert st["round1"] == "bucketed" and st["passes"][0] == 2, st


@pytest.mark.parametrize("round1", ["lsd", "bucketed"])
def test_round1_variants_agree(gpu, oracle, round1):
    """Both first-round sorts give the same round-1 groups (D_1, unsorted
    count) and the same SA, including the sparse-rank look-ups of later
    rounds through the bucketed key layout."""
    from hpc_suffix_array_amd import build_suffix_array
    for kind, n in (("dna", 3_000_017), ("alnum", 1_500_007), ("byte256", 1 << 21)):
        t = oracle.gen_text(kind, n, seed=n)
        got, st = build_suffix_array(t, return_stats=True, round1=round1)
        # the same K for both (auto K: the bucketed round takes the fewest
        # symbols, the LSD round rounds K up to whole radix passes)
        ref, st_ref = build_suffix_array(t, return_stats=True, round1="lsd", init_chars=st["init_chars"])
        assert (got == ref).all() and (got == oracle.sa_c(t)).all(), (kind, round1)
        assert st["round1"] == round1
        assert st["distinct"] == st_ref["distinct"], (kind, st["distinct"], st_ref["distinct"])


def test_bucketed_round1_fallback(gpu, oracle):
    """Skewed texts overflow a window (one bucket > the LDS tile): the first
    round falls back to the full LSD sort and the SA stays exact."""
    from hpc_suffix_array_amd import build_suffix_array
    n = 1 << 20
    for t in (np.full(n, ord("a"), np.uint8),
              np.tile(np.frombuffer(b"abaababa", np.uint8), n // 8),
              np.concatenate([oracle.gen_text("dna", n // 2, seed=3), np.full(n // 2, ord("C"), np.uint8)])):
        got, st = build_suffix_array(t, return_stats=True, round1="bucketed")
        # one symbol: all but the last K suffixes share suffix 0's key -> the
        # LSD round's pivot split (pivot_round1)
        assert st["round1"] == ("pivot" if len(np.unique(t)) == 1 else "lsd"), st["round1"]
        if len(np.unique(t)) > 1:   # one symbol: no bucketing at all (sigma < 2)
            assert st["largest_window"] > 18432, st["largest_window"]
        assert (got == oracle.sa_c(t)).all()


def test_pivot_round1(gpu, oracle):
    """The LSD round 1 split around suffix 0's key (pivot_round1, sa_pivot.h
    R1) when half or more of the suffixes share it: a long run of one symbol
    before random text, one symbol with sparse noise (the rest above the
    pivot, the text's last suffixes below it), ragged sizes; a text whose
    suffix 0 key is rare keeps the LSD sort.  Same SA as the oracle and as the full LSD sort (debug no_pivot)."""
    from hpc_suffix_array_amd import build_suffix_array
    rng = np.random.default_rng(5)
    cases = [(np.concatenate([np.full(700_001, ord("a"), np.uint8), oracle.gen_text("dna", 300_000, seed=1)]),
              "pivot"),
             (np.where(rng.random(600_000) < 0.001, ord("b"), ord("a")).astype(np.uint8), "pivot"),
             (np.concatenate([np.full(65_600, ord("z"), np.uint8), rng.integers(97, 100, 999, dtype=np.uint8)]),
              "pivot"),
             (np.concatenate([oracle.gen_text("dna", 300_000, seed=2), np.full(700_000, ord("a"), np.uint8)]),
              "lsd")]
    for t, want in cases:
        got, st = build_suffix_array(t, return_stats=True, round1="lsd")
        assert st["round1"] == want, (len(t), st["round1"])
        assert (got == oracle.sa_c(t)).all(), len(t)
        ref = build_suffix_array(t, round1="lsd", debug=("no_pivot",))
        assert (got == ref).all()


def test_bucketed_round1_known_answers(gpu, oracle, golden):
    """The default (auto) path at 1 MiB and 64 MiB takes the bucketed first
    round; SHA-256 known answers of SURVEY.md 8(c)."""
    from hpc_suffix_array_amd import build_suffix_array
    for key in ("alnum_1MiB", "ascii127_1MiB", "dna_1MiB", "byte256_1MiB", "dna_64MiB"):
        k = golden["known"][key]
        t = oracle.gen_text(k["kind"], k["n"], seed=k["seed"])
        got, st = build_suffix_array(t, return_stats=True)
        assert st["round1"] == "bucketed", key
        assert oracle.sha256(got.astype(np.int32)) == k["sa_sha256_i32"], key


def test_bucketed_round1_dense_ranks(gpu, oracle):
    """A repeated random block: the bucketed first round leaves almost every
    suffix unsorted, so the later rounds keep dense ranks and read every
    sorted key1 -- the local sort runs again writing all of them (the sparse
    path keeps only every 16th, sa_round1.h kKeySample)."""
    from hpc_suffix_array_amd import build_suffix_array
    block = oracle.gen_text("dna", 100_003, seed=11)
    t = np.concatenate([np.tile(block, 20), oracle.gen_text("dna", 1001, seed=12)])
    got, st = build_suffix_array(t, return_stats=True, round1="bucketed")
    assert st["round1"] == "bucketed" and not st["sparse_ranks"], st
    assert (got == oracle.sa_c(t)).all()
    # random text of the same size: sparse ranks through the key samples
    t = oracle.gen_text("dna", len(t), seed=13)
    got, st = build_suffix_array(t, return_stats=True, round1="bucketed")
    assert st["round1"] == "bucketed" and st["sparse_ranks"], st
    assert (got == oracle.sa_c(t)).all()


@pytest.mark.parametrize("mode", ["padded", "overflow", "exact"])
def test_round1_padded_segments(gpu, oracle, golden, mode):
    """From 2^26 suffixes the first bucket pass writes into segments sized
    from a 1-in-2^ssh sample (k_bucket_sample, sa_bucket.h) instead of exact
    digit totals; a segment that overflows (forced here by debug
    "pad_overflow": no slack) makes the round run again with the exact
    totals; "no_pad" takes the exact totals at once.  Config-2 known answer
    (64 MiB DNA) through all three."""
    from hpc_suffix_array_amd import build_suffix_array
    dbg = {"padded": (), "overflow": ("pad_overflow",), "exact": ("no_pad",)}[mode]
    k = golden["known"]["dna_64MiB"]
    t = oracle.gen_text(k["kind"], k["n"], seed=k["seed"])
    got, st = build_suffix_array(t, return_stats=True, debug=dbg)
    assert st["round1"] == "bucketed"
    assert st["round1_segments"] == {"padded": "padded", "overflow": "padded-overflow", "exact": "exact"}[mode], st
    assert oracle.sha256(got.astype(np.int32)) == k["sa_sha256_i32"]


def test_round1_padded_segments_skewed(gpu, oracle):
    """Padded segments on texts whose first-pass digits are far from uniform
    (a biased alphabet: digit sizes ~2x apart; a long random block repeated):
    exact SA either way
    (an overflow falls back to the exact totals)."""
    from hpc_suffix_array_amd import build_suffix_array, check_suffix_array
    n = (1 << 26) + 12345
    rng = np.random.default_rng(5)
    biased = rng.choice(np.frombuffer(b"ACGT", np.uint8), size=n, p=[0.3, 0.3, 0.2, 0.2])
    got, st = build_suffix_array(biased, return_stats=True)
    assert st["round1"] == "bucketed" and st["round1_segments"] in ("padded", "padded-overflow"), st
    assert (got == oracle.sa_c(biased)).all()
    # a long random block repeated (dense ranks; the oracle's 20+ rounds over
    # 64 M suffixes would take minutes: the O(n) checker instead)
    block = oracle.gen_text("alnum", 3_000_017, seed=9)
    rep = np.tile(block, n // len(block) + 1)[:n]
    got, st = build_suffix_array(rep, return_stats=True)
    assert st["round1"] == "bucketed" and st["round1_segments"] in ("padded", "padded-overflow"), st
    assert check_suffix_array(rep, got)


@pytest.mark.parametrize("layout", ["default", "no_pk8", "no_cmp"])
def test_round1_layouts(gpu, oracle, golden, layout):
    """Key layouts of the bucketed first round (sa_kernels.h BucketSpec,
    sa_split.h k_split_text<.., PK8>): the compact low (cmp) with packed
    8-byte first-pass items (pk8, wherever the bits fit: sa_round1.h
    plan_pk8), the compact low alone, and the original layout -- same SA."""
    from hpc_suffix_array_amd import build_suffix_array
    dbg = () if layout == "default" else (layout,)
    for kind, n in (("dna", 3_000_017), ("byte256", 1 << 21), ("alnum", 1_500_007), ("binary", 1 << 20)):
        t = oracle.gen_text(kind, n, seed=n + 1)
        t[-1] = t.max()   # no tail run of the smallest symbol (test_compact_layout_text_tails)
        got, st = build_suffix_array(t, return_stats=True, round1="bucketed", debug=dbg)
        assert st["round1"] == "bucketed", (kind, st)
        lay = st["round1_layout"]
        assert lay["compact"] == (layout != "no_cmp"), (kind, lay)
        if layout == "no_pk8":
            assert not lay["pk8"], (kind, lay)
        elif kind != "binary":   # alnum (sigma 62) through the fraction form of D - Dmin(bucket)
            assert lay["pk8"], (kind, lay)
        assert (got == oracle.sa_c(t)).all(), (kind, layout)
    if layout == "default":   # config 2 through the packed items (1 GiB: the bench)
        k = golden["known"]["dna_64MiB"]
        t = oracle.gen_text(k["kind"], k["n"], seed=k["seed"])
        got, st = build_suffix_array(t, return_stats=True)
        # 2^26 suffixes: 16-bit buckets of ~1024 suffixes, below the fixed-span
        # local sort's 4 window strides, so the second pass takes one region
        assert st["round1_layout"] == {"compact": True, "pk8": True, "xq": False, "eonly": False}, st["round1_layout"]
        assert oracle.sha256(got.astype(np.int32)) == k["sa_sha256_i32"]


@pytest.mark.parametrize("tail", [b"A" * 40, b"CAA", b"ACGTACGTTTGCA" * 3, b"T" * 40, b"GATTACA"])
def test_compact_layout_text_tails(gpu, oracle, tail):
    """The compact key1 low is exact only when no two of the text's last
    K - 1 suffixes share (D, r) (sa_round1.h short_suffix_ties): a text
    ending in a run of its smallest symbol breaks that and takes the original
    layout;
    other tails keep the compact one.  Same SA as the oracle either way."""
    from hpc_suffix_array_amd import build_suffix_array
    n = 1 << 21
    t = np.concatenate([oracle.gen_text("dna", n - len(tail), seed=len(tail)), np.frombuffer(tail, np.uint8)])
    got, st = build_suffix_array(t, return_stats=True)
    assert st["round1"] == "bucketed"
    smallest_run = tail.endswith(b"AA")   # "A" and "AA" pad alike
    assert st["round1_layout"]["compact"] == (not smallest_run), (tail, st["round1_layout"])
    assert (got == oracle.sa_c(t)).all()


@pytest.mark.parametrize("kind", ["alnum", "ascii127", "dna", "binary"])
def test_eonly_layout(gpu, oracle, kind):
    """The E-only key1 layout (BucketSpec.cmp = 2, no end bit: what lets 1 GiB
    alnum / ascii127 pack their first-pass items) forced at every size: short
    suffixes share keys with the suffixes continuing them with the smallest
    symbol and round 2 orders them.  Texts whose last K suffixes pad alike
    (a tail run of the smallest symbol) must keep the compact layout.  Also
    the packed non-power-of-two items (np2 PK8, k_bucket_dmin) on their own."""
    from hpc_suffix_array_amd import build_suffix_array
    for n in (70_001, 1 << 20, 3_000_017):
        t = oracle.gen_text(kind, n, seed=n + 5)
        want = oracle.sa_c(t)
        got, st = build_suffix_array(t, return_stats=True, round1="bucketed", debug=("eonly",))
        assert (got == want).all(), (kind, n)
        assert st["round1"] == "bucketed", (kind, n)
        if kind != "binary":   # (a random binary tail often pads alike: compact / original layout, still exact)
            assert st["round1_layout"]["eonly"], (kind, n, st["round1_layout"])
        got, st = build_suffix_array(t, return_stats=True, round1="bucketed")
        assert (got == want).all(), (kind, n)
        if kind in ("alnum", "ascii127"):   # non-power-of-two items packed at these sizes (compact layout fits)
            assert st["round1_layout"]["pk8"], (kind, n, st["round1_layout"])
        # tails that defeat the E-only precondition: the smallest symbol repeated
        tt = t.copy()
        tt[-(st["init_chars"] + 3):] = tt.min()
        got, st = build_suffix_array(tt, return_stats=True, round1="bucketed", debug=("eonly",))
        assert (got == oracle.sa_c(tt)).all(), (kind, n, "tail")
        assert not st["round1_layout"]["eonly"], (kind, n)
        # one short suffix equal to the smallest symbol only (passes the check
        # when the rest of the tail differs): "...x" + smallest
        tt = t.copy()
        tt[-1] = t.min()
        got, st = build_suffix_array(tt, return_stats=True, round1="bucketed", debug=("eonly",))
        assert (got == oracle.sa_c(tt)).all(), (kind, n, "one")


def test_local_sort_variants(gpu):
    """The fixed-span local sort's variants (sa_bucket.h k_bucket_sort LSV,
    sa_opts.tune bits 16-19): unconditional network reads, suffix indices
    written back by the sorting threads (the U walk converting the
    sub-buckets with groups), both -- each with per-XCD chunks (XQ) and with
    one region (no_xq), on random DNA and on DNA with a planted repeat (groups
    left by round 1 in many windows); same SA as the default, O(n)-checked."""
    import torch
    from hpc_suffix_array_amd import DeviceBuilder
    n = (1 << 28) + 4097
    b = DeviceBuilder(n)
    t = torch.empty(n, dtype=torch.uint8, device="cuda")
    want = torch.empty(n, dtype=torch.int32, device="cuda")
    got = torch.empty(n, dtype=torch.int32, device="cuda")
    try:
        for kind in ("dna", "repeats"):
            b.generate_text(t, n, b"ACGT", seed=11)
            if kind == "repeats":   # ~4 K 64-symbol blocks each copied once: pairs of equal 20-symbol keys
                ar = torch.arange(64, device="cuda")[None, :]
                src = torch.arange(0, n - 70_000, 65_536, device="cuda")[:, None] + ar
                t[(src + 32_768).reshape(-1)] = t[src.reshape(-1)]
            t[-1] = ord("T")
            for dbg in ((), ("no_xq",)):
                st0 = b.build(t, n, want, debug=dbg)
                assert st0["round1"] == "bucketed", st0
                assert b.check(t, n, want), (kind, dbg)
                for v in (1, 2, 3, 4):
                    b.build(t, n, got, debug=dbg, tune=v << 16)
                    assert bool((got == want).all().item()), (kind, dbg, v)
    finally:
        b.close()


def test_round1_xq_second_pass(gpu):
    """The second bucket pass by per-XCD queues and regions (sa_split.h
    k_split_seg<.., XQ>, k_bucket_starts_xq; sa_bucket.h load_items_xq,
    k_window_gather) against the one-region pass (debug no_xq), at 2^28 + 4097
    suffixes (the smallest size whose buckets take the fixed-span local sort):
    packed DNA items, a DNA text with "TT" made rare (uneven buckets: windows
    of several buckets go through k_window_gather) and sub-regions without slack
    (xq_overflow: a queue overflows, the round runs again with one region);
    alnum and a widened span take one region at this size.  Same SA in every
    case, O(n)-checked.  (1 GiB DNA, the bench, and the slow 2^30 - 1 known
    answer run the XQ pass too.)"""
    import torch
    from hpc_suffix_array_amd import DeviceBuilder
    n = (1 << 28) + 4097
    b = DeviceBuilder(n)
    t = torch.empty(n, dtype=torch.uint8, device="cuda")
    want = torch.empty(n, dtype=torch.int32, device="cuda")
    got = torch.empty(n, dtype=torch.int32, device="cuda")
    try:
        for kind, alpha in (("dna", b"ACGT"), ("alnum", bytes(range(48, 58)) + bytes(range(65, 91)) + bytes(range(97, 123))),
                            ("rare_tt", b"ACGT")):
            b.generate_text(t, n, alpha, seed=7)
            if kind == "rare_tt":   # "TT" made rare: buckets of TT-prefixes hold ~3 %, windows span several
                g = torch.Generator(device="cuda").manual_seed(3)
                tt = (t[1:] == ord("T")) & (t[:-1] == ord("T")) & (torch.rand(n - 1, device="cuda", generator=g) < 0.97)
                repl = torch.tensor(list(b"ACG"), dtype=torch.uint8, device="cuda")[
                    torch.randint(0, 3, (n - 1,), device="cuda", generator=g)]
                t[1:] = torch.where(tt, repl, t[1:])
                del tt, repl
            t[-1] = max(alpha)   # no tail run of the smallest symbol (compact layout)
            st0 = b.build(t, n, want, debug=("no_xq",))
            assert not st0["round1_layout"]["xq"] and st0["round1"] == "bucketed", (kind, st0["round1_layout"])
            assert b.check(t, n, want), kind
            # (alnum at this size: buckets below 4 window strides, one region;
            # span_extra 6: the span no longer fits the fixed-span words)
            for dbg, extra, xq in (((), 0, kind != "alnum" or None), ((), 6, None), (("xq_overflow",), 0, False)):
                st = b.build(t, n, got, debug=dbg, span_extra=extra)
                print(kind, dbg, extra, st["round1_layout"], flush=True)
                assert xq is None or st["round1_layout"]["xq"] == xq, (kind, dbg, extra, st["round1_layout"])
                assert bool((got == want).all().item()), (kind, dbg, extra)
    finally:
        b.close()


@pytest.mark.parametrize("extra", [0, 6])
def test_local_sort_fixed_span(gpu, oracle, extra):
    """One-bucket windows of the compact layout split the bucket's whole key
    span into sub-buckets without measuring it (sa_bucket.h load_window,
    SA_LS_FIXED_SPAN); a window whose keys cluster (forced here by a span 2^6
    too wide: every key in the lowest sub-buckets) is listed for a second
    launch that measures its span (sa_round1.h, retry list) instead of going
    to the LSD kernel."""
    from hpc_suffix_array_amd import build_suffix_array
    for kind, n in (("dna", 3_000_017), ("byte256", 1 << 21)):
        t = oracle.gen_text(kind, n, seed=n + 5)
        t[-1] = t.max()
        got, st = build_suffix_array(t, return_stats=True, round1="bucketed", span_extra=extra)
        assert st["round1"] == "bucketed" and st["round1_layout"]["compact"], (kind, st)
        assert (got == oracle.sa_c(t)).all(), (kind, extra)


@pytest.mark.slow
@pytest.mark.gpu
def test_config4_partition_at_its_own_shape(gpu):
    """configs[3] at its own shape, played rank by rank on one GPU: byte256
    text of n = 2^32 suffixes over G = 8 ranks (19-bit buckets, 32-bit index
    fields, ~2^29 suffixes per rank).  The cut plan covers n suffixes in
    contiguous SA ranges, every rank's round 1 sorts its slice on the first K
    symbols, the slices follow each other in SA order and every text position
    lands in exactly one slice (scripts/sim_ranks.py --check; the later
    rounds' look-ups across ranks are the multi-rank tests' and the 8-GPU
    run's)."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import sim_ranks
    rows = sim_ranks.simulate(1 << 32, "byte256", [8], ranks="all", reps=0, check=True)
    assert len(rows) == 8 and all(r["checked"] and r["ok"] == 1 for r in rows)
    assert sum(r["m"] for r in rows) == 1 << 32
    assert max(r["share"] for r in rows) < 1.2, rows
    assert rows[0]["bucket_bits"] == 19


# configs[3] (4 GiB byte256 over 8 GPUs, manber_myers_mpi.c:108-144) at the
# largest shape one MI355X holds as several ranks: n = 2^31 + 17 over 4 HIP
# ranks (~2^29 suffixes each, 32-bit index fields, 18-19-bit buckets), with
# copies of one 3000-byte block planted across the text so that groups survive
# round 1 and the later rounds' rank look-ups cross ranks for several rounds.
CFG4_N = (1 << 31) + 17
CFG4_PLANT = (1000, 3000, 7)   # source offset, block length, copies


def _cfg4_text(ops, torch):
    n = CFG4_N
    t = torch.empty(n, dtype=torch.uint8, device="cuda")
    ops.b.generate_text(t, n, bytes(range(256)), seed=3)
    src, L, copies = CFG4_PLANT
    blk = t[src: src + L].clone()
    for k in range(1, copies + 1):
        p = k * (n // (copies + 1)) + 777
        t[p: p + L] = blk
    torch.cuda.synchronize()
    return t


def _cfg4_log(name):
    import faulthandler
    logdir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(logdir, exist_ok=True)
    log = open(os.path.join(logdir, f"cfg4_{name}.log"), "w")
    os.dup2(log.fileno(), 2)
    os.environ["SA_DIST_TRACE"] = "1"
    faulthandler.dump_traceback_later(150, exit=True, file=log)
    return lambda *a: print(*a, file=log, flush=True)


def _cfg4_reference(port, path, q):
    """World-1 build of the planted text through the same driver (the path
    test_distributed_hip_config4_shape pins), O(n)-checked, its SA written to
    host shared memory for the ranks' slice comparison; this process exits
    before the ranks start, so its HBM is free again."""
    sys.path.insert(0, ROOT)
    say = _cfg4_log("reference")
    import torch
    import torch.distributed as dist
    from hpc_suffix_array_amd.distributed import DistributedSA, HipRangeOps
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
        ops = HipRangeOps(0, 0)
        t = _cfg4_text(ops, torch)
        d = DistributedSA(ops)
        sa_local, sa_off = d.build(t, CFG4_N)
        torch.cuda.synchronize()
        say("built", d.stats)
        ok = bool(ops.b.check(t, CFG4_N, sa_local))
        say("checked", ok)
        mm = np.memmap(path, dtype=np.int32, mode="w+", shape=(CFG4_N,))
        step = 1 << 27
        for a in range(0, CFG4_N, step):
            b = min(CFG4_N, a + step)
            mm[a:b] = sa_local[a:b].cpu().numpy()
        mm.flush()
        del mm
        say("written")
        q.put({"ok": ok, "path": d.stats["path"], "m": d.stats["m"], "rounds": d.stats["rounds"],
               "unsorted": d.stats["unsorted"]})
    except BaseException:
        import traceback
        say(traceback.format_exc())
        q.put({"error": traceback.format_exc()})
        raise
    finally:
        dist.destroy_process_group()


def _cfg4_rank(rank, world, port, path, q):
    """One of `world` HIP ranks sharing the box's GPU (collectives staged
    through gloo): the range-partitioned build, then this rank's SA slice
    against the same slice of the world-1 build."""
    sys.path.insert(0, ROOT)
    say = _cfg4_log(f"w{world}_r{rank}")
    import torch
    import torch.distributed as dist
    from hpc_suffix_array_amd.distributed import DistributedSA, HipRangeOps
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        ops = HipRangeOps(0, 0)
        t = _cfg4_text(ops, torch)
        d = DistributedSA(ops)
        sa_local, sa_off = d.build(t, CFG4_N)
        torch.cuda.synchronize()
        say("built", d.stats)
        m = sa_local.numel()
        ref = np.memmap(path, dtype=np.int32, mode="r", shape=(CFG4_N,))
        want = torch.from_numpy(np.array(ref[int(sa_off): int(sa_off) + m])).cuda()   # a writable host copy
        eq = bool((want == sa_local).all().item())
        say("compared", eq)
        free, _ = torch.cuda.mem_get_info()
        q.put({"rank": rank, "eq": eq, "m": m, "sa_off": int(sa_off), "path": d.stats["path"],
               "free_gib": free / (1 << 30), "round1_ms": d.stats["phase_ms"].get("round1"),
               "rounds": d.stats["rounds"], "requests": d.stats["requests"],
               "cross": d.stats["cross_requests"], "bucket_bits": d.stats["bucket_bits"]})
    except BaseException:
        import traceback
        say(traceback.format_exc())
        q.put({"rank": rank, "error": traceback.format_exc()})
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.slow
def test_config4_cross_rank_rounds_eight_and_four_ranks(gpu):
    """configs[3]'s range partition end to end at n = 2^31 + 17 byte256 over
    8 ranks (configs[3]'s own world size) and then 4 ranks, all on the box's
    GPU: round 1 per range and every later round's rank requests and answers
    exchanged between ranks (sa_dist_req_* / sa_dist_answer / sa_dist_refine
    and the sliced all-to-alls of distributed.py), each rank's SA slice equal
    to the O(n)-checked world-1 build of the same text
    (manber_myers_mpi.c:108-144 is the shape replaced; the 8-GPU RCCL run is
    the driver's).  HBM: ~26 GiB per rank at 8 ranks (text 2 GiB, the
    n-bit member map and its prefix 0.5 GiB, ~90 B per suffix of the
    ~2^28-suffix range), ~210 GiB in all."""
    import gc
    import socket

    import torch
    import torch.multiprocessing as mp
    gc.collect()
    torch.cuda.empty_cache()   # this process's cached HBM (earlier tests) back to the device
    shm = "/dev/shm" if os.path.isdir("/dev/shm") else "/tmp"
    path = os.path.join(shm, f"sa_cfg4_{os.getpid()}.i32")

    def port():
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            return s.getsockname()[1]

    ctx = mp.get_context("spawn")
    try:
        q = ctx.Queue()
        p = ctx.Process(target=_cfg4_reference, args=(port(), path, q))
        p.start()
        ref = q.get(timeout=300)
        p.join(timeout=60)
        assert "error" not in ref, ref["error"]
        assert p.exitcode == 0
        assert ref["ok"] and ref["path"] == "range" and ref["m"] == CFG4_N, ref
        for world in (8, 4):
            pt = port()
            procs = [ctx.Process(target=_cfg4_rank, args=(r, world, pt, path, q)) for r in range(world)]
            for pr in procs:
                pr.start()
            res = sorted((q.get(timeout=300) for _ in range(world)), key=lambda x: x["rank"])
            for pr in procs:
                pr.join(timeout=60)
            errs = [x["error"] for x in res if "error" in x]
            assert not errs, (world, errs[0])
            assert all(pr.exitcode == 0 for pr in procs)
            assert all(x["path"] == "range" for x in res), res
            assert all(x["eq"] for x in res), (world, [(x["rank"], x["eq"]) for x in res])
            # the ranges tile the SA in rank order
            off = 0
            for x in res:
                assert x["sa_off"] == off, res
                off += x["m"]
            assert off == CFG4_N
            assert max(x["m"] for x in res) < 1.2 * CFG4_N / world, (world, [x["m"] for x in res])
            # later rounds with look-ups answered by other ranks: at least two
            cross = res[0]["cross"]
            assert sum(1 for c in cross if c > 0) >= 2, res[0]
            assert res[0]["rounds"] >= 3 and ref["rounds"] >= 3, (res[0], ref)
            print(f"world {world}: m {[x['m'] for x in res]}, rounds {res[0]['rounds']}, cross {cross}, "
                  f"HBM free after the builds {min(x['free_gib'] for x in res):.1f} GiB, "
                  f"round1 ms {[x['round1_ms'] for x in res]}", flush=True)
    finally:
        if os.path.exists(path):
            os.remove(path)
