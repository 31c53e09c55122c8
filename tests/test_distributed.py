"""Multi-rank paths under gloo on CPU: the range-partitioned
driver (DistributedSA) and its sample-sort fallback (SampleSortSA) with the
CPU stand-ins of their local operations (tests/dist_cpu_ops.py), world sizes
2 and 3, checked against the oracle.  The same drivers run with the HIP
phases + RCCL on the GPU box (tests/test_gpu_parity.py::test_distributed_*
and bench.py --gpus N)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _texts():
    import sys
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    return {
        "dna": O.gen_text("dna", 20_011, seed=3),
        "binary": O.gen_text("binary", 9_001, seed=4),
        "byte256": O.gen_text("byte256", 7_000, seed=5),
        "degenerate": np.full(1_500, ord("a"), np.uint8),
        "periodic": np.tile(np.frombuffer(b"abaababa", np.uint8), 700),
        "tiny1": np.frombuffer(b"x", np.uint8),
        "tiny2": np.frombuffer(b"ba", np.uint8),
        "banana": np.frombuffer(b"banana", np.uint8),
    }


def _worker(rank, world, port, q, chunks=None, driver="range", piece=None):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    from dist_cpu_ops import CpuOps, CpuRangeOps
    from hpc_suffix_array_amd import distributed as D
    from hpc_suffix_array_amd.distributed import DistributedSA, SampleSortSA, gather_sa
    if chunks:
        D.XCHUNK, D.CHUNK = chunks
    if piece:
        D.TEXT_PIECE = piece
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = {}
        for name, t in _texts().items():
            text = torch.from_numpy(t.copy())
            if driver == "range":
                d = DistributedSA(CpuRangeOps())
                sa_local, sa_off = d.build(text, len(t))
            elif driver == "sliced":
                # rank r starts from its slice only; the build gathers the rest
                C = D.text_chunk(len(t), world)
                sl = text[min(len(t), rank * C): min(len(t), (rank + 1) * C)].clone()
                del text
                d = DistributedSA(CpuRangeOps())
                sa_local, sa_off = d.build_sliced(sl, len(t))
            else:
                d = SampleSortSA(CpuOps())
                sa_local, sa_off = d.build(text, len(t)), len(t) * rank // world
            sa = gather_sa(sa_local, sa_off, len(t))
            res[name] = (sa.numpy(), d.stats)
        if rank == 0:
            q.put(res)
    finally:
        dist.destroy_process_group()


def _run(oracle, world, chunks=None, driver="range", piece=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, chunks, driver, piece)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for name, t in _texts().items():
        sa, st = res[name]
        want = oracle.sa_c(t)
        assert (sa == want.astype(np.int64)).all(), (name, world, driver)
        if driver in ("range", "sliced"):
            # one repeated symbol (sigma = 1) has no bucket layout: sample sort
            want_path = "sample-sort" if len(np.unique(t)) < 2 else "range"
            assert st["path"] == want_path, (name, st)
            if want_path == "range":
                assert st["unsorted"][-1] == 0, (name, st)
        else:
            assert st["distinct"][-1] == len(t), name
    return res


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_gloo(oracle, world):
    """The range-partitioned driver: bucket-range cuts, local first rounds,
    rank requests / answers by all_to_all, several doubling rounds (K = 3)."""
    res = _run(oracle, world)
    assert max(len(st["unsorted"]) for _, st in res.values()) >= 3


@pytest.mark.parametrize("world", [2, 3])
def test_distributed_gloo_sliced(oracle, world):
    """The N > 1 bench's input: rank r holds only text[r C, (r + 1) C); the
    build gathers the text (one all_gather, inside the build) and agrees on
    failures at the collectives it needs anyway.  Pins the collectives and
    host read-backs per build: text gather 1 + alphabet 1 + coarse 1 + per
    round one count gather (+ two exchanges in every round but the last);
    read-backs: alphabet 1 + coarse 1 + one per round."""
    res = _run(oracle, world, driver="sliced")
    for name, (_, st) in res.items():
        if st["path"] != "range":
            continue
        R = len(st["unsorted"])   # count gathers (the last finds nothing unsorted)
        assert st["collectives"] == 3 + R + 2 * (R - 1), (name, st)
        assert st["host_syncs_driver"] == 2 + R, (name, st)
        assert st["host_syncs_native"] == 0 and st["host_syncs"] == st["host_syncs_driver"]


def test_distributed_gloo_sliced_pieces(oracle):
    """The text gathered in pieces (TEXT_PIECE tiny: configs[3]'s 4 GiB path)."""
    _run(oracle, 3, driver="sliced", piece=3000)


def _fail_worker(rank, world, port, q, where):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    from dist_cpu_ops import CpuRangeOps
    from hpc_suffix_array_amd.distributed import DistributedSA

    class Failing(CpuRangeOps):
        rounds = 0

        def begin(self, *a):
            if where == "begin" and rank == 1:
                raise MemoryError("injected begin failure")
            return super().begin(*a)

        def answer(self, req):
            if where == "answer" and rank == 0:
                raise RuntimeError("injected answer failure")
            return super().answer(req)

        def refine(self, h, ans, sa_local):
            Failing.rounds += 1
            if where == "refine" and rank == world - 1 and Failing.rounds == 2:
                raise RuntimeError("injected refine failure")
            return super().refine(h, ans, sa_local)

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t = _texts()["periodic"]
        try:
            DistributedSA(Failing()).build(torch.from_numpy(t.copy()), len(t))
            q.put((rank, "ok"))
        except Exception as e:   # noqa: BLE001
            q.put((rank, type(e).__name__ + ": " + str(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("where", ["begin", "answer", "refine"])
def test_distributed_failure_agreement(where):
    """A phase failing on one rank makes every rank raise at the build's next
    collective (the failing rank its own error), instead of leaving the others
    blocked: no per-phase agreement collective is needed."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 3
    procs = [ctx.Process(target=_fail_worker, args=(r, world, port, q, where)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    failing = {"begin": 1, "answer": 0, "refine": world - 1}[where]
    for rank, msg in got.items():
        assert msg != "ok", got
        if rank == failing:
            assert "injected" in msg, got
        else:
            assert "another rank" in msg, got


@pytest.mark.parametrize("world", [2, 3])
def test_sample_sort_gloo(oracle, world):
    """The sample-sort fallback driver (skewed texts)."""
    _run(oracle, world, driver="sample")


def _plan(sa_lib, world, bb, hist):
    import ctypes
    h = np.ascontiguousarray(hist, dtype=np.uint64)
    cuts = np.zeros(world + 1, np.uint32)
    mmax = ctypes.c_uint64()
    rc = sa_lib.lib().sa_dist_plan_cuts(world, int(h.sum()), bb, h.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                        cuts.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), ctypes.byref(mmax))
    return rc, cuts, int(mmax.value)


def test_dist_cut_plan(sa_lib):
    """sa_dist_plan_cuts (host only): at 19-bit buckets a range holds at most
    2048 coarse buckets (2^18 local buckets).  A balanced text whose midpoint
    falls just past coarse bucket 2048 at W = 2 (the 2^31+17 config-4 shape)
    must be clamped to 2048 | 2048, not planned 2049 | 2047 and reported
    unbalanced."""
    hist = np.full(4096, 1000, np.uint64)
    hist[0], hist[2048] = 0, 2000           # prefix at 2048 just below n / 2
    rc, cuts, mmax = _plan(sa_lib, 2, 19, hist)
    assert rc == 0 and list(cuts) == [0, 2048, 4096] and mmax == 2049000
    # uniform at every world size: equal ranges, contiguous, within the cap
    for world in (1, 2, 3, 4, 8):
        for bb in (16, 17, 18, 19):
            rc, cuts, mmax = _plan(sa_lib, world, bb, np.full(4096, 7, np.uint64))
            cap = (1 << 18) >> (bb - 12)
            if world * cap < 4096:   # the ranges cannot cover the buckets (plan_bucketed never asks)
                assert rc == 2
                continue
            assert rc == 0, (world, bb)
            assert cuts[0] == 0 and cuts[-1] == 4096 and (np.diff(cuts.astype(np.int64)) >= 0).all()
            assert (np.diff(cuts.astype(np.int64)) <= cap).all()
            assert mmax <= 7 * (4096 // world + 1)
    # the nearer boundary: prefix 4999 vs 5001 around n / 2 = 5000 (W = 2)
    hist = np.zeros(4096, np.uint64)
    hist[:10] = [1000, 1000, 1000, 1000, 999, 1001, 1000, 1000, 1000, 1000]
    rc, cuts, mmax = _plan(sa_lib, 2, 16, hist)
    assert rc == 0 and cuts[1] == 5 and mmax == 5001
    # one coarse bucket holding most suffixes cannot balance
    hist = np.ones(4096, np.uint64)
    hist[7] = 10_000_000
    rc, cuts, _ = _plan(sa_lib, 4, 16, hist)
    assert rc == 2
    # a histogram that does not sum to n is an argument error
    import ctypes
    h = np.ones(4096, np.uint64)
    cuts = np.zeros(3, np.uint32)
    m = ctypes.c_uint64()
    assert sa_lib.lib().sa_dist_plan_cuts(2, 5, 16, h.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                          cuts.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), ctypes.byref(m)) < 0


def test_choose_chars_keeps_int64_keys():
    from hpc_suffix_array_amd.distributed import choose_chars
    for sigma in (1, 2, 3, 4, 26, 62, 127, 255, 256):
        K, base = choose_chars(sigma, 1 << 30)
        assert base ** K <= 1 << 63 and K >= 1
    assert choose_chars(4, 1 << 30) == (20, 5)


def test_chunked_helpers(monkeypatch):
    """chunked_map (the sample-sort driver's elementwise steps over slices)
    agrees with the unsliced op."""
    import torch
    from hpc_suffix_array_amd import distributed as D
    monkeypatch.setattr(D, "CHUNK", 7)
    g = torch.Generator().manual_seed(3)
    for n in (0, 1, 6, 7, 8, 50):
        mask = torch.rand(n, generator=g) < 0.4
        x = torch.randint(-5, 40, (n,), generator=g)
        assert torch.equal(D.chunked_map(lambda m, v: torch.where(m, v, -1), mask, x), torch.where(mask, x, -1))


def test_distributed_gloo_sliced_exchange(oracle):
    """The sliced all_to_all_v / all_gather paths (XCHUNK, CHUNK tiny)."""
    _run(oracle, 3, chunks=(97, 1000))
    _run(oracle, 2, chunks=(97, 1000), driver="sample")


def test_exchange_slice_limit():
    """The all_to_all slice bound the exchanges rely on: one all_to_all_single
    of 2^28 int64 (2 GiB) returned half garbage on this ROCm stack, so every
    collective moves at most XCHUNK elements per peer pair -- below 2^31 bytes
    for the widest payload (int64) -- and gather_sa's all_gather slices stay
    below 2^31 bytes per rank too."""
    from hpc_suffix_array_amd import distributed as D
    assert D.XCHUNK * 8 < (1 << 31)
    assert D.CHUNK * 8 < (1 << 31)
    # the 1 GiB DNA build's request exchange at G = 2 (~0.5 M int32 per peer)
    # and the sample-sort fallback's bucket exchange at 2^30 / 8 ranks (2^27
    # int64 per peer) are sliced into 1 and 4 collectives
    assert -(-(1 << 19) // D.XCHUNK) == 1 and -(-(1 << 27) // D.XCHUNK) == 4


def _summary_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    import bench
    from dist_cpu_ops import CpuRangeOps
    from hpc_suffix_array_amd.distributed import DistributedSA
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t = _texts()["periodic"]
        d = DistributedSA(CpuRangeOps())
        d.build(torch.from_numpy(t.copy()), len(t))
        st = dict(d.stats)
        # CPU stand-ins have no HIP events: per-rank phase and round-1 kernel
        # times as a GPU rank would report them (rank 1 the slower)
        st["phase_ms"] = {"alphabet": 0.1, "round1": 2.0 + rank, "requests": 0.5, "exchange": 0.2}
        m = st["m"]
        kern = {"scatter_keys": {"ms": 1.0 + rank, "launches": 1, "bytes": 16 * m},
                "local_sort": {"ms": 0.5, "launches": 1, "bytes": 12 * m},
                "scan": {"ms": 5.0, "launches": 3, "bytes": 0}}
        rec = bench.rank_record(rank, [st], kern)
        recs = [None] * world
        dist.all_gather_object(recs, rec)
        if rank == 0:
            q.put((recs, bench.distributed_summary(recs, len(t)), len(t)))
    finally:
        dist.destroy_process_group()


def test_bench_distributed_summary_gloo():
    """bench.py's N > 1 fields (per-rank roofline of the slowest rank's
    dominant round-1 kernel, per-rank round-1 GB/s, phase times max over
    ranks, xGMI bytes per later round) from the records of a world-2 gloo
    build of the range-partitioned driver (the RCCL run gathers the same
    records with all_gather_object)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_summary_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    recs, s, n = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r["rank"] for r in recs] == [0, 1]
    assert sum(r["m"] for r in recs) == n and recs[1]["sa_off"] == recs[0]["m"]
    roof = s["roofline"]
    m1 = recs[1]["m"]
    # rank 1 has the slower round 1; its dominant kernel (scan excluded) is
    # scatter_keys: 16 m bytes in 2.0 ms
    assert roof["rank"] == 1 and roof["kind"] == "scatter_keys", roof
    assert roof["bytes_per_launch"] == 16 * m1 and roof["avg_launch_ms"] == 2.0
    assert abs(roof["achieved"] - 16 * m1 / 2e-3 / 1e9) < 0.1
    assert abs(roof["frac"] - roof["achieved"] / 8000.0) < 1e-4
    assert roof["unit"] == "GB/s" and roof["bound"] == "hbm" and roof["peak"] == 8000.0
    pr = s["round1_per_rank"]
    assert [x["round1_ms"] for x in pr] == [2.0, 3.0]
    assert pr[0]["round1_bytes"] == 28 * recs[0]["m"]
    assert s["kernels_ms_per_step"]["round1"] == 3.0 and s["kernels_ms_per_step"]["requests"] == 0.5
    assert s["kernels_ms_per_step"]["round1_kernels_slowest_rank"]["scatter_keys"] == 2.0
    # the periodic text needs later rounds; some look-ups cross ranks
    cross = s["cross_requests_per_round"]
    assert len(cross) >= 2 and any(c > 0 for c in cross)
    assert s["xgmi_bytes_per_round"] == [12 * c for c in cross]
    assert s["requests_per_round"] == recs[0]["requests"]
    assert abs(s["largest_rank_share"] - max(r["m"] for r in recs) / (n / 2)) < 1e-3
