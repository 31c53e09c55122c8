"""Range-partitioned multi-GPU suffix-array build.

One process per GPU (torch.distributed; backend "nccl" is RCCL over xGMI on
MI355X, "gloo" for the CPU tests).  Every rank holds the text in HBM (1 byte
per suffix -- the reference's MPI driver broadcasts it too, main_mpi.c:51);
the suffix array and all working state are split into G contiguous SA
ranges.  The product path is ``DistributedSA`` over ``HipRangeOps`` (the
sa_dist_* phases of libsa_hip, include/sa_hip.h):

  alphabet   each rank's slice -> all_reduce MAX of the 256 presence flags
  begin      K and the bucket plan (bucket = the first s symbols); coarse
             bucket histogram of the rank's text slice
  cuts       all_reduce SUM of the coarse histograms -> every rank derives
             the same G contiguous bucket ranges of ~n/G suffixes; rank q's
             suffixes occupy SA positions [sa_off_q, sa_off_q + m_q)
  round 1    each rank scans its text copy, keeps the suffixes of its bucket
             range and sorts them by their first K symbols (bucket passes +
             per-window LDS sort): no records cross xGMI
  round h    while any rank has unsorted suffixes (all_gather of counts):
             rank[x + h] requests to the rank owning x + h's bucket
             (all_to_all), answers back (all_to_all), local sort of the
             unsorted set by (group, rank[x + h]) and re-rank -- groups never
             straddle ranks, so only rank look-ups cross the links

This replaces the reference's MPI strategy (src/mpi/manber_myers_mpi.c:
108-144: qsort per rank, Gatherv of all records to rank 0, serial qsort
there, Bcast of the whole rank array every round), which is centralised and
does not scale.  Texts whose buckets cannot balance (one repeated symbol,
very short periods) fall back to ``SampleSortSA`` (all ranks agree through a
collective).

The same drivers run under gloo on CPU with CPU stand-ins of the local
operations in tests/ (test infrastructure); the product path fails loudly
without the HIP library.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from . import _native as N

I64 = torch.int64
I32 = torch.int32
SAMPLES = 64
# torch's index / scan kernels are used on slices of at most CHUNK elements:
# on 2^30-element tensors (1 GiB, world size 1) torch.bincount raised SIGFPE
# and an index_put faulted on ROCm; permutations go through HIP kernels
CHUNK = 1 << 26
# elements per peer pair in one all_to_all_single (see alltoallv)
XCHUNK = 1 << 25
COARSE = 4096   # coarse buckets of the cut plan (sa_bucket.h kCoarse)


# -- collectives shared by both drivers -----------------------------------------
# gloo has no device collectives: with a gloo group and HIP tensors (several
# ranks sharing one GPU -- the multi-rank HIP tests of tests/test_gpu_parity.py)
# each collective is staged through host memory; RCCL groups use HBM directly.
def _staged(t: torch.Tensor, group) -> bool:
    return t.is_cuda and dist.get_backend(group) == "gloo"


def _all_reduce(t: torch.Tensor, op=dist.ReduceOp.SUM, group=None) -> None:
    if _staged(t, group):
        h = t.cpu()
        dist.all_reduce(h, op=op, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op, group=group)


def _all_gather(out: List[torch.Tensor], t: torch.Tensor, group=None) -> None:
    if _staged(t, group):
        ho = [torch.empty_like(x, device="cpu") for x in out]
        dist.all_gather(ho, t.cpu(), group=group)
        for x, y in zip(out, ho):
            x.copy_(y)
    else:
        dist.all_gather(out, t, group=group)


def _all_to_all_single(out: torch.Tensor, inp: torch.Tensor, rs=None, ss=None, group=None) -> None:
    if _staged(inp, group):
        ho = torch.empty_like(out, device="cpu")
        dist.all_to_all_single(ho, inp.cpu(), rs, ss, group=group)
        out.copy_(ho)
    else:
        dist.all_to_all_single(out, inp, rs, ss, group=group)


def _all_gather_into(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    """out = the ranks' equal-size inputs back to back, in rank order
    (RCCL all_gather_into_tensor: no copy; gloo: rows of out)."""
    G = dist.get_world_size(group)
    if _staged(inp, group):
        ho = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather(list(ho.view(G, -1).unbind(0)), inp.cpu(), group=group)
        out.copy_(ho)
    elif dist.get_backend(group) == "gloo":
        dist.all_gather(list(out.view(G, -1).unbind(0)), inp, group=group)
    else:
        dist.all_gather_into_tensor(out, inp, group=group)


# bytes of text one all_gather moves in total at most: larger texts (configs[3],
# 4 GiB) are gathered in pieces (a 2 GiB all_to_all_single returned garbage on
# this ROCm stack, see alltoallv)
TEXT_PIECE = 1 << 30


def text_chunk(n: int, world: int) -> int:
    """Symbols per rank of the input partition: rank r holds
    text[r C, min(n, (r + 1) C)) with C = ceil(n / world) (n / world each when
    it divides, as every bench size does)."""
    return -(-n // world) if world > 0 else n


def alltoallv(tensors: List[torch.Tensor], send: List[int], recv: Optional[List[int]] = None,
              group=None, slices: Optional[int] = None) -> Tuple[List[torch.Tensor], List[int]]:
    """all_to_all_v of each tensor (send[j] elements to rank j, in rank order).
    Each collective moves at most XCHUNK elements per peer pair: one
    all_to_all_single of 2^28 int64 (2 GiB) returned half garbage on this
    ROCm stack, so larger exchanges run in slices, the slice count agreed by a
    MAX all_reduce (tests/test_distributed.py pins the sliced path)."""
    G = dist.get_world_size(group)
    if G == 1:
        return list(tensors), list(send)
    dev = tensors[0].device
    if recv is None:
        sc = torch.tensor(send, dtype=I64, device=dev)
        rc = torch.empty_like(sc)
        _all_to_all_single(rc, sc, group=group)
        recv = rc.tolist()
    C = XCHUNK
    if slices is None:   # the slice count, agreed by every rank
        t_loc = torch.tensor([max([0] + [(x + C - 1) // C for x in list(send) + list(recv)])], dtype=I64, device=dev)
        _all_reduce(t_loc, op=dist.ReduceOp.MAX, group=group)
        T = int(t_loc.item())
    else:                # known to every rank already (e.g. from an all_gathered count matrix)
        T = int(slices)
    so = [sum(send[:j]) for j in range(G)]
    ro = [sum(recv[:j]) for j in range(G)]
    outs = []
    for t in tensors:
        t = t.contiguous()
        o = torch.empty(sum(recv), dtype=t.dtype, device=dev)
        if T <= 1:
            _all_to_all_single(o, t, list(recv), list(send), group=group)
            outs.append(o)
            continue
        for k in range(T):
            sl = [min(C, max(0, x - k * C)) for x in send]
            rl = [min(C, max(0, x - k * C)) for x in recv]
            inp = torch.cat([t[so[j] + k * C: so[j] + k * C + sl[j]] for j in range(G)])
            got = torch.empty(sum(rl), dtype=t.dtype, device=dev)
            _all_to_all_single(got, inp, rl, sl, group=group)
            a = 0
            for j in range(G):
                o[ro[j] + k * C: ro[j] + k * C + rl[j]] = got[a: a + rl[j]]
                a += rl[j]
        outs.append(o)
    return outs, list(recv)


def _all_gather_rows(row: torch.Tensor, group=None) -> List[List[int]]:
    G = dist.get_world_size(group)
    if G == 1:
        return [row.tolist()]
    out = [torch.empty_like(row) for _ in range(G)]
    _all_gather(out, row.contiguous(), group=group)
    return torch.stack(out).cpu().tolist()


def _present_words(flags: Sequence[int]) -> List[int]:
    words = [0] * 8
    for b in range(256):
        if flags[b]:
            words[b >> 5] |= 1 << (b & 31)
    return words


# -- product local operations: libsa_hip's sa_dist_* phases -------------------------
class HipRangeOps:
    """One rank's local phases of the range-partitioned build on its GPU
    (include/sa_hip.h sa_dist_*; kernels in csrc/sa_dist.h)."""

    def __init__(self, max_n: int, device: int, world: Optional[int] = None):
        from .builder import DeviceBuilder
        self.dev = torch.device("cuda", device)
        self.b = DeviceBuilder(0, device=device)
        self.L = N.lib()
        self.info = N.SaDistInfo()
        self.coarse = torch.zeros(COARSE, dtype=I64, device=self.dev)
        self.round1_stats = N.SaStats()
        self.profile = False
        self.textbuf = None
        if world:   # everything a build allocates, ahead of the first one
            N.check(self.L.sa_dist_reserve(self.b.ctx, max_n, world), "sa_dist_reserve")
            # the gathered text: world equal chunks (DistributedSA.build_sliced)
            self.textbuf = torch.empty(world * text_chunk(max_n, world), dtype=torch.uint8, device=self.dev)

    def host_syncs(self) -> int:
        """Host waits libsa_hip has made so far (sa_host_syncs)."""
        return int(self.L.sa_host_syncs())

    def _s(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)

    def _info(self) -> dict:
        i = self.info
        return {k: getattr(i, k) for k, _ in N.SaDistInfo._fields_}

    def alphabet(self, text_slice: torch.Tensor) -> List[int]:
        out = (ctypes.c_uint32 * 8)()
        if text_slice.numel():
            N.check(self.L.sa_alphabet_device(text_slice.data_ptr(), text_slice.numel(), out, self._s()),
                    "sa_alphabet_device")
        return list(out)

    def begin(self, text: torch.Tensor, n: int, world: int, rank: int, present: Sequence[int]):
        self.text = text
        pw = (ctypes.c_uint32 * 8)(*present)
        N.check(self.L.sa_dist_begin(self.b.ctx, text.data_ptr(), n, world, rank, pw, self.coarse.data_ptr(),
                                     self._s(), ctypes.byref(self.info)), "sa_dist_begin")
        return self._info(), self.coarse

    def cuts(self, coarse_host: Optional[torch.Tensor]) -> dict:
        if coarse_host is None:
            N.check(self.L.sa_dist_cuts(self.b.ctx, None, ctypes.byref(self.info)), "sa_dist_cuts")
        else:
            h = coarse_host.to(I64).contiguous().numpy().astype("uint64")
            N.check(self.L.sa_dist_cuts(self.b.ctx, h.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)),
                                        ctypes.byref(self.info)), "sa_dist_cuts")
        return self._info()

    def empty(self, m: int, dtype) -> torch.Tensor:
        return torch.empty(m, dtype=dtype, device=self.dev)

    def round1(self, sa_local: torch.Tensor) -> dict:
        st = ctypes.byref(self.round1_stats) if self.profile else None
        N.check(self.L.sa_dist_round1(self.b.ctx, sa_local.data_ptr() if sa_local.numel() else None, self._s(),
                                      ctypes.byref(self.info), st), "sa_dist_round1")
        return self._info()

    def req_count(self, h: int, world: int) -> Tuple[List[int], dict]:
        c = (ctypes.c_uint64 * world)()
        N.check(self.L.sa_dist_req_count(self.b.ctx, h, c, self._s(), ctypes.byref(self.info)), "sa_dist_req_count")
        return [int(x) for x in c], self._info()

    def req_fill(self, h: int, nsend: int) -> torch.Tensor:
        req = torch.empty(nsend, dtype=I32, device=self.dev)
        N.check(self.L.sa_dist_req_fill(self.b.ctx, h, req.data_ptr() if nsend else None, self._s()),
                "sa_dist_req_fill")
        return req

    def answer(self, req: torch.Tensor) -> torch.Tensor:
        ans = torch.empty(req.numel(), dtype=I64, device=self.dev)
        if req.numel():
            N.check(self.L.sa_dist_answer(self.b.ctx, req.data_ptr(), req.numel(), ans.data_ptr(), self._s()),
                    "sa_dist_answer")
        return ans

    def refine(self, h: int, ans: torch.Tensor, sa_local: torch.Tensor) -> dict:
        N.check(self.L.sa_dist_refine(self.b.ctx, h, ans.data_ptr() if ans.numel() else None,
                                      sa_local.data_ptr() if sa_local.numel() else None, self._s(),
                                      ctypes.byref(self.info)), "sa_dist_refine")
        return self._info()

    def fallback_ops(self) -> "HipOps":
        """The sample-sort driver's operations on this rank's own context:
        the range build's per-rank buffers (n-entry rank array, member map,
        request buffers) are released first and the workspace is shared, so
        the fallback does not double the HBM footprint."""
        N.check(self.L.sa_dist_release(self.b.ctx), "sa_dist_release")
        if not hasattr(self, "_fb"):
            self._fb = HipOps(0, self.dev.index, builder=self.b)
        return self._fb


def _trace(*a):
    import os
    import sys
    if os.environ.get("SA_DIST_TRACE"):
        print("[dist]", *a, file=sys.stderr, flush=True)


class DistributedSA:
    """Range-partitioned build over an initialised process group.

    ``build_sliced(text_slice, n)`` -> (sa_local, sa_off): the input as
    north_star partitions it -- rank r holds only text[r C, (r + 1) C) (C =
    text_chunk(n, G)) -- gathered to every rank by one RCCL all_gather (part
    of the build, as the reference times its text MPI_Bcast,
    main_mpi.c:40-51), then the build.  ``build(text, n)`` starts from the
    whole text on every rank.  sa_local is this rank's slice of the SA, SA
    positions [sa_off, sa_off + len(sa_local)) (uint32 values stored as
    int32 by the HIP path; int64 from the sample-sort fallback).

    Failure agreement rides on the collectives the build needs anyway: a
    phase that raises on one rank (a libsa_hip SAError -- NOMEM, a request
    outside the range --, a torch OOM, ...) is recorded, the rank carries on
    with placeholder buffers of the agreed sizes, and its error flag travels
    in the next all_reduce / all_gather of the build (the alphabet flags, the
    coarse histogram, the per-round count rows), where every rank raises --
    no extra collective or host wait per phase.  So are the range plan's
    fallback decisions (unbalanced cuts, a window over the LDS tile).
    stats: "collectives" and "host_syncs" per build (the driver's reads of
    device data and blocking uploads, plus libsa_hip's own waits)."""

    def __init__(self, ops, group=None):
        self.ops = ops
        self.group = group
        self.G = dist.get_world_size(group)
        self.r = dist.get_rank(group)
        self.stats = {}

    def _mark(self, name: str, dev) -> None:
        """HIP event on the build stream at a phase boundary (stats["phase_ms"])."""
        if dev.type != "cuda":
            return
        e = torch.cuda.Event(enable_timing=True)
        e.record(torch.cuda.current_stream(dev))
        self._events.append((name, e))

    def _phase_ms(self) -> dict:
        out = {}
        if len(self._events) > 1:
            self._events[-1][1].synchronize()
            self._syncs += 1
            for (a, ea), (_, eb) in zip(self._events, self._events[1:]):
                out[a] = round(out.get(a, 0.0) + ea.elapsed_time(eb), 4)
        return out

    # -- failure agreement and counting --------------------------------------
    def _run(self, name: str, fn, *args, default=None):
        """One local phase; at G > 1 an exception is recorded (raised at the
        next agreement point) and `default` stands in for the result."""
        try:
            return fn(*args)
        except Exception as e:   # noqa: BLE001 -- agreed on, then re-raised
            if self.G == 1:
                raise
            if self._err is None:
                self._err = (name, e)
            _trace("phase failed", name, e)
            return default() if callable(default) else default

    def _raise_agreed(self, flagged: bool) -> None:
        """An agreement point: some rank flagged an error -> every rank raises
        (the failing rank its own exception)."""
        if self._err is not None:
            raise self._err[1]
        if flagged:
            raise N.SAError("sa_dist: a phase failed on another rank")

    def _coll(self, fn, *args, **kw):
        self._ncoll += 1
        return fn(*args, **kw)

    def _to_host(self, t: torch.Tensor) -> List:
        self._syncs += 1   # a device read-back on the GPU (counted on CPU too: the same program points)
        return t.cpu().tolist()

    @staticmethod
    def _upload(vals: List[int], dev, dtype=I64) -> torch.Tensor:
        """A small row on the device through a pinned host buffer, without a
        host wait (torch keeps the buffer until the copy has run)."""
        if dev.type != "cuda":
            return torch.tensor(vals, dtype=dtype)
        return torch.tensor(vals, dtype=dtype).pin_memory().to(dev, non_blocking=True)

    def _reset(self) -> None:
        self.stats = {"path": "range", "rounds": 0, "unsorted": [], "requests": [], "cross_requests": []}
        self._events = []
        self._err = None
        self._ncoll = 0
        self._syncs = 0
        self._native0 = self.ops.host_syncs() if hasattr(self.ops, "host_syncs") else 0

    def _finish(self) -> None:
        native = (self.ops.host_syncs() - self._native0) if hasattr(self.ops, "host_syncs") else 0
        self.stats["collectives"] = self._ncoll
        self.stats["host_syncs_driver"] = self._syncs
        self.stats["host_syncs_native"] = native
        self.stats["host_syncs"] = self._syncs + native

    # -- the input partition ----------------------------------------------------
    def gather_text(self, text_slice: torch.Tensor, n: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """The whole text on every rank from the ranks' slices (rank r:
        text[r C, min(n, (r + 1) C)), C = text_chunk(n, G)) by all_gather into
        `out` (>= G C bytes; allocated when None); slices of more than
        TEXT_PIECE / G bytes are gathered piecewise."""
        G, r = self.G, self.r
        C = text_chunk(n, G)
        want = min(n, (r + 1) * C) - min(n, r * C)
        if text_slice.numel() != want:
            raise ValueError(f"rank {r} holds {text_slice.numel()} symbols, the partition gives it {want}")
        if G == 1:
            return text_slice
        dev = text_slice.device
        if out is None or out.numel() < G * C:
            out = torch.empty(G * C, dtype=torch.uint8, device=dev)
        P = max(1, TEXT_PIECE // G)
        if C <= P:
            send = text_slice
            if want < C:   # the last ranks' short slices, padded
                send = torch.zeros(C, dtype=torch.uint8, device=dev)
                send[:want] = text_slice
            self._coll(_all_gather_into, out[: G * C], send, self.group)
            return out[:n]
        view = out[: G * C].view(G, C)
        for a in range(0, C, P):
            b = min(C, a + P)
            send = torch.zeros(b - a, dtype=torch.uint8, device=dev)
            e = min(b, want)
            if e > a:
                send[: e - a] = text_slice[a:e]
            got = torch.empty(G * (b - a), dtype=torch.uint8, device=dev)
            self._coll(_all_gather_into, got, send, self.group)
            view[:, a:b] = got.view(G, b - a)
        return out[:n]

    def build_sliced(self, text_slice: torch.Tensor, n: int, out: Optional[torch.Tensor] = None):
        self._reset()
        dev = text_slice.device
        self._mark("text_gather", dev)
        text = self.gather_text(text_slice, n, out if out is not None else getattr(self.ops, "textbuf", None))
        return self._build(text, n)

    def build(self, text: torch.Tensor, n: int):
        self._reset()
        return self._build(text, n)

    # -- the build ----------------------------------------------------------------
    def _build(self, text: torch.Tensor, n: int):
        G, r = self.G, self.r
        dev = text.device
        lo, hi = n * r // G, n * (r + 1) // G
        self._mark("alphabet", dev)
        # alphabet of the whole text: OR of the slices' masks (MAX of flags;
        # the NCCL backend has no bitwise-or reduction); flag 256 = an error
        _trace("alphabet", r, G, n)
        words = self._run("alphabet", self.ops.alphabet, text[lo:hi], default=[0] * 8)
        flags = self._upload([(words[b >> 5] >> (b & 31)) & 1 for b in range(256)] + [1 if self._err else 0], dev,
                             I32)
        if G > 1:
            self._coll(_all_reduce, flags, op=dist.ReduceOp.MAX, group=self.group)
        fl = self._to_host(flags)
        self._raise_agreed(bool(fl[256]))
        present = _present_words(fl[:256])
        if n < 2:
            return self._fallback(text, n, "n < 2")
        _trace("begin")
        self._mark("begin", dev)
        res = self._run("begin", self.ops.begin, text, n, G, r, present)
        info, coarse = res if res is not None else (None, None)
        ch = None
        if G > 1:
            # the coarse histograms summed, with the begin phase's error flag
            self._mark("coarse_allreduce", dev)
            agg = torch.zeros(COARSE + 1, dtype=I64, device=dev)
            if coarse is not None:
                agg[:COARSE] = coarse.to(dev)
            if self._err is not None:
                agg[COARSE] = 1
            self._coll(_all_reduce, agg, group=self.group)
            self._syncs += 1
            ch = agg.cpu()
            self._raise_agreed(bool(ch[COARSE]))
            ch = ch[:COARSE]
        self.stats.update(sigma=info["sigma"], K=info["K"], bucket_bits=info["bucket_bits"])
        if info["status"] != N.DIST_OK:   # identical on every rank (global alphabet and n)
            return self._fallback(text, n, "unsupported alphabet / size")
        _trace("cuts")
        self._mark("cuts", dev)   # the cut plan (the workspace: reserved by HipRangeOps(max_n, device, world))
        info = self._run("cuts", self.ops.cuts, ch)
        fallback = None
        sa_local = None
        if info is not None:
            _trace("cut", info)
            self.stats.update(m=info["m"], sa_off=info["sa_off"], m_max=info["m_max"])
            if info["status"] != N.DIST_OK:   # identical on every rank (same global histogram)
                fallback = "unbalanced bucket ranges"
            else:
                self._mark("sa_local", dev)
                sa_local = self._run("sa_local", self.ops.empty, info["m"], I32)
                if sa_local is not None:
                    self._mark("round1", dev)
                    info = self._run("round1", self.ops.round1, sa_local)
                    _trace("round1", info)
                    if info is not None and info["round1_ok"] == 0:
                        fallback = "a bucket window exceeds the LDS tile"
        self.stats["rounds"] = 1
        if info is not None and "heads" in info:
            self.stats["heads_round1"] = info["heads"]
        h = self.stats.get("K") or 1
        first = True
        while True:
            # the round's one agreement point: every rank's [error, fallback,
            # unsorted, requests per owner], gathered by all ranks
            self._mark("requests", dev)
            counts, uns = [0] * G, 0
            if self._err is None and fallback is None:
                res = self._run("req_count", self.ops.req_count, h, G)
                if res is not None:
                    counts, info = res
                    uns = info["unsorted"]
            _trace("req_count", h, counts)
            row = [1 if self._err else 0, 1 if fallback else 0, uns] + counts
            mat = self._gather_rows(self._upload(row, dev))
            self._raise_agreed(any(x[0] for x in mat))
            if any(x[1] for x in mat):
                if not first:
                    raise RuntimeError("sa_dist: fallback requested after round 1")
                return self._fallback(text, n, fallback or "a bucket window exceeds the LDS tile on another rank")
            first = False
            total_u = sum(x[2] for x in mat)
            self.stats["unsorted"].append(total_u)
            if total_u == 0:
                break
            if h >= 2 * n:
                raise RuntimeError("distributed doubling did not converge")
            recv_counts = [x[3 + r] for x in mat]
            self.stats["requests"].append(sum(sum(x[3:]) for x in mat))
            # look-ups answered by another rank (they cross xGMI under RCCL)
            self.stats["cross_requests"].append(sum(x[3 + q] for p, x in enumerate(mat) for q in range(G) if q != p))
            # every rank holds the whole count matrix: the slice count of both
            # exchanges needs no extra collective
            slices = max([0] + [(y + XCHUNK - 1) // XCHUNK for x in mat for y in x[3:]])
            nreq = sum(counts)
            req = self._run("req_fill", self.ops.req_fill, h, nreq,
                            default=lambda: torch.zeros(nreq, dtype=I32, device=dev))
            self._mark("exchange", dev)
            (got,), _ = self._alltoallv([req], counts, recv_counts, slices)
            _trace("requests in", got.numel())
            self._mark("answer", dev)
            ans = self._run("answer", self.ops.answer, got,
                            default=lambda: torch.zeros(got.numel(), dtype=I64, device=dev))
            self._mark("exchange", dev)
            (back,), _ = self._alltoallv([ans], recv_counts, counts, slices)
            self._mark("refine", dev)
            if self._err is None:
                self._run("refine", self.ops.refine, h, back, sa_local)
            _trace("refined", h)
            self.stats["rounds"] += 1
            h *= 2
        self._mark("end", dev)
        self.stats["phase_ms"] = self._phase_ms()
        self._finish()
        return sa_local, self.stats["sa_off"]

    def _gather_rows(self, row: torch.Tensor) -> List[List[int]]:
        if self.G == 1:
            return [self._to_host(row)]
        out = [torch.empty_like(row) for _ in range(self.G)]
        self._coll(_all_gather, out, row.contiguous(), group=self.group)
        return self._to_host(torch.stack(out))

    def _alltoallv(self, tensors, send, recv, slices):
        if self.G == 1:
            return list(tensors), list(send)
        T = max(1, int(slices))
        self._ncoll += T * len(tensors)
        return alltoallv(tensors, send, recv, self.group, slices)

    def _fallback(self, text, n, why):
        self.stats["path"] = "sample-sort"
        self.stats["fallback_reason"] = why
        ops = self.ops.fallback_ops()
        d = SampleSortSA(ops, self.group)
        sa = d.build(text, n)
        self.stats.update(d.stats)
        self.stats["path"] = "sample-sort"
        self._finish()
        return sa, n * self.r // self.G


def gather_sa(sa_local: torch.Tensor, sa_off: int, n: int, group=None) -> torch.Tensor:
    """The full SA (int64) on every rank from the ranks' contiguous slices
    (any sizes); all_gathers of at most CHUNK elements per rank."""
    G = dist.get_world_size(group)
    if G == 1:
        return sa_local.to(I64) if sa_local.dtype != I32 else (sa_local.to(I64) & 0xFFFFFFFF)
    dev = sa_local.device
    loc = sa_local.to(I64)
    if sa_local.dtype == I32:
        loc = loc & 0xFFFFFFFF
    rows = _all_gather_rows(torch.tensor([int(sa_off), loc.numel()], dtype=I64, device=dev), group)
    m = max(x[1] for x in rows)
    buf = torch.full((max(m, 1),), -1, dtype=I64, device=dev)
    buf[: loc.numel()] = loc
    full = torch.full((n,), -1, dtype=I64, device=dev)
    for a in range(0, max(m, 1), CHUNK):
        b = min(max(m, 1), a + CHUNK)
        out = [torch.empty(b - a, dtype=I64, device=dev) for _ in range(G)]
        _all_gather(out, buf[a:b].contiguous(), group=group)
        for q, (off, cnt) in enumerate(rows):
            e = min(b, cnt)
            if e > a:
                full[off + a: off + e] = out[q][: e - a]
    return full


def chunked_map(fn, *ts: torch.Tensor) -> torch.Tensor:
    """fn applied elementwise over CHUNK-element slices of equal-length
    vectors: torch's own kernels never see 2^30 elements here (bincount and
    index_put faulted at that size on ROCm)."""
    m = ts[0].numel()
    if m <= CHUNK:
        return fn(*ts)
    return torch.cat([fn(*(t[a: a + CHUNK] for t in ts)) for a in range(0, m, CHUNK)])


def bit_width(x: int) -> int:
    return int(x).bit_length()


def choose_chars(sigma: int, n: int, limit_bits: int = 63) -> Tuple[int, int]:
    """(K, base) for the packed first key, as sa_build.hip choose_chars but
    with base^K <= 2^limit_bits so keys stay non-negative int64."""
    base = sigma + 1
    kmax = 0
    while base ** (kmax + 1) <= (1 << limit_bits):
        kmax += 1
    if sigma <= 1:
        return max(kmax, 1), base
    kmin = 1
    while sigma ** kmin < 512 * n and kmin < kmax:
        kmin += 1
    passes = (bit_width(base ** kmin - 1) + 7) // 8
    K = kmin
    while K + 1 <= kmax and bit_width(base ** (K + 1) - 1) <= 8 * passes:
        K += 1
    return K, base


class HipOps:
    """Local per-rank operations on the GPU through libsa_hip's C ABI."""

    def __init__(self, max_n: int, device: int, builder=None):
        from .builder import DeviceBuilder
        self.dev = torch.device("cuda", device)
        self.b = builder if builder is not None else DeviceBuilder(max_n, device=device)
        self.L = N.lib()

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)

    def alphabet(self, text: torch.Tensor) -> List[int]:
        out = (ctypes.c_uint32 * 8)()
        N.check(self.L.sa_alphabet_device(text.data_ptr(), text.numel(), out, self._stream()), "sa_alphabet_device")
        return list(out)

    def pack_keys(self, text: torch.Tensor, n: int, lo: int, hi: int, codes: Sequence[int], base: int,
                  K: int) -> torch.Tensor:
        keys = torch.empty(hi - lo, dtype=I64, device=self.dev)
        if hi == lo:   # an empty slice (n < world size)
            return keys
        code = (ctypes.c_uint16 * 256)(*codes)
        N.check(self.L.sa_pack_keys_device(self.b.ctx, text.data_ptr(), n, lo, hi, code, base, K, keys.data_ptr(),
                                           self._stream()), "sa_pack_keys_device")
        return keys

    def argsort(self, keys: torch.Tensor, bits: int) -> Tuple[torch.Tensor, torch.Tensor]:
        m = keys.numel()
        if m == 0:
            return keys, torch.empty(0, dtype=I64, device=keys.device)
        vals = torch.arange(m, dtype=torch.int32, device=keys.device)
        ko = torch.empty_like(keys)
        vo = torch.empty_like(vals)
        N.check(self.L.sa_sort_pairs_device(self.b.ctx, keys.data_ptr(), vals.data_ptr(), m, max(bits, 1),
                                            ko.data_ptr(), vo.data_ptr(), self._stream()), "sa_sort_pairs_device")
        return ko, vo.to(I64)

    def gather(self, src: torch.Tensor, idx: torch.Tensor, base: int = 0) -> torch.Tensor:
        """src[idx - base] (int64) by a HIP kernel (torch's index kernels are
        avoided on 2^30-element tensors, see scatter)."""
        assert src.dtype == I64 and idx.dtype == I64
        src, idx = src.contiguous(), idx.contiguous()
        out = torch.empty(idx.numel(), dtype=I64, device=idx.device)
        N.check(self.L.sa_gather_u64_device(out.data_ptr(), src.data_ptr(), src.numel(), idx.data_ptr(), base,
                                            idx.numel(), self._stream()), "sa_gather_u64_device")
        return out

    def running_max(self, v: torch.Tensor) -> torch.Tensor:
        """Inclusive running max (int64) by HIP kernels: torch.cummax took
        3.1 s of a 3.4 s distributed build at 1 GiB."""
        assert v.dtype == I64
        out = v.contiguous().clone()
        N.check(self.L.sa_running_max_i64_device(out.data_ptr(), out.numel(), self._stream()),
                "sa_running_max_i64_device")
        return out

    def scatter(self, dst: torch.Tensor, idx: torch.Tensor, base: int, src: torch.Tensor) -> None:
        """dst[idx - base] = src (int64) by a HIP kernel: torch's index_put
        faulted on the GPU for 2^30-element int64 targets (1 GiB, world 1)."""
        assert dst.dtype == I64 and idx.dtype == I64 and src.dtype == I64 and idx.numel() == src.numel()
        idx, src = idx.contiguous(), src.contiguous()
        N.check(self.L.sa_scatter_u64_device(dst.data_ptr(), dst.numel(), idx.data_ptr(), base, src.data_ptr(),
                                             idx.numel(), self._stream()), "sa_scatter_u64_device")

    def count_below(self, sorted_x: torch.Tensor, q: torch.Tensor, right: bool = False) -> torch.Tensor:
        """For each q the number of elements of the sorted (non-negative)
        int64 vector below q (at most q with right): a binary search per
        query (sa_count_below_u64_device)."""
        sorted_x, q = sorted_x.contiguous(), q.contiguous()
        out = torch.empty(q.numel(), dtype=I64, device=q.device)
        if q.numel():
            N.check(self.L.sa_count_below_u64_device(sorted_x.data_ptr() if sorted_x.numel() else None,
                                                     sorted_x.numel(), q.data_ptr(), q.numel(), 1 if right else 0,
                                                     out.data_ptr(), self._stream()), "sa_count_below_u64_device")
        return out

    def cumsum(self, x: torch.Tensor) -> torch.Tensor:
        """Inclusive int64 prefix sum (sa_inclusive_sum_i64_device)."""
        out = x.to(I64).contiguous().clone()
        N.check(self.L.sa_inclusive_sum_i64_device(out.data_ptr(), out.numel(), self._stream()),
                "sa_inclusive_sum_i64_device")
        return out

    def select(self, mask: torch.Tensor) -> torch.Tensor:
        """int64 positions of the set elements of a bool vector, in order
        (sa_select_u8_device: per-tile counts, their scan, ordered writes).
        The output is sized by a counting call first, so the result holds
        exactly its elements (an m-entry buffer behind a view would keep 8m
        bytes alive while the caller holds the selection)."""
        mask = mask.contiguous()
        total = self.count_true(mask)
        out = torch.empty(total, dtype=I64, device=mask.device)
        if total == 0:
            return out
        cnt = ctypes.c_uint64()
        N.check(self.L.sa_select_u8_device(mask.data_ptr() if mask.numel() else None, mask.numel(),
                                           out.data_ptr(), ctypes.byref(cnt), self._stream()), "sa_select_u8_device")
        if cnt.value != total:
            raise N.SAError(f"sa_select_u8_device: {cnt.value} selected after a count of {total}")
        return out

    def count_true(self, mask: torch.Tensor) -> int:
        """Number of set elements of a bool vector (one device count, one sync)."""
        mask = mask.contiguous()
        cnt = ctypes.c_uint64()
        N.check(self.L.sa_select_u8_device(mask.data_ptr() if mask.numel() else None, mask.numel(), None,
                                           ctypes.byref(cnt), self._stream()), "sa_select_u8_device")
        return int(cnt.value)


class SampleSortSA:
    """General range-partitioned builder by sample sort (the fallback of
    DistributedSA for texts whose bucket ranges cannot balance: one repeated
    symbol, very short periods).  Rank r owns text positions and SA positions
    [r n / G, (r+1) n / G); round 1 sorts packed K-symbol keys globally
    (local radix sort, G*64 (key, rank, position) splitters, all_to_all_v of
    the buckets, local re-sort), later rounds fetch rank[i + h] from its
    position owner and sort the unsorted set globally by (group, rank)."""

    def __init__(self, ops, group=None):
        self.ops = ops
        self.group = group
        self.G = dist.get_world_size(group)
        self.r = dist.get_rank(group)
        self.stats = {}

    # -- collectives ---------------------------------------------------------
    def _gather(self, t: torch.Tensor) -> torch.Tensor:
        out = [torch.empty_like(t) for _ in range(self.G)]
        _all_gather(out, t.contiguous(), group=self.group)
        return torch.stack(out)

    def _sum(self, x: int, dev) -> int:
        t = torch.tensor([x], dtype=I64, device=dev)
        _all_reduce(t, group=self.group)
        return int(t.item())

    def _alltoallv(self, tensors: List[torch.Tensor], send: List[int]) -> Tuple[List[torch.Tensor], List[int]]:
        return alltoallv(tensors, send, None, self.group)

    def _route(self, dest: torch.Tensor, tensors: List[torch.Tensor]):
        # destination order by the local HIP radix sort (stable), counts by
        # searching the sorted destinations: torch.bincount over 2^30
        # elements raised SIGFPE on ROCm (1 GiB, world size 1)
        if self.G == 1:   # everything stays: no permutation, no exchange
            order = torch.arange(dest.numel(), dtype=I64, device=dest.device)
            return list(tensors), [dest.numel()], order, [dest.numel()]
        else:
            sd, order = self.ops.argsort(dest.to(I64), bit_width(self.G - 1))
            q = torch.arange(self.G + 1, dtype=I64, device=dest.device)
            send = torch.diff(self.ops.count_below(sd, q)).tolist()
        outs, recv = self._alltoallv([self.ops.gather(t, order) for t in tensors], send)
        return outs, recv, order, send

    # -- sorting ---------------------------------------------------------------
    def _dist_sort(self, keys: torch.Tensor, payloads: List[torch.Tensor], bits: int):
        """Global stable sort by key (order of equal keys: source rank, then
        source position).  Returns sorted keys/payloads of this rank's
        segment and the segment's global offset."""
        dev = keys.device
        keys, perm = self.ops.argsort(keys, bits)
        payloads = [self.ops.gather(p, perm) for p in payloads]
        m = keys.numel()
        if self.G == 1:   # the local sort is the global one
            return keys, payloads, 0, [m]
        # samples (key, rank, position, valid)
        s = min(SAMPLES, m)
        samp = torch.zeros(SAMPLES, 4, dtype=I64, device=dev)
        if s:
            pos = torch.arange(s, dtype=I64, device=dev) * m // s
            samp[:s, 0] = keys[pos]
            samp[:s, 1] = self.r
            samp[:s, 2] = pos
            samp[:s, 3] = 1
        allsamp = self._gather(samp).reshape(-1, 4).cpu()
        allsamp = allsamp[allsamp[:, 3] == 1].tolist()
        allsamp.sort()
        cuts = []
        for j in range(1, self.G):
            if not allsamp:
                cuts.append(m)
                continue
            ks, rs, ps, _ = allsamp[min(len(allsamp) - 1, j * len(allsamp) // self.G)]
            kt = torch.tensor([ks], dtype=I64, device=dev)
            lo = int(self.ops.count_below(keys, kt).item())
            hi = int(self.ops.count_below(keys, kt, right=True).item())
            if self.r < rs:
                c = hi
            elif self.r > rs:
                c = lo
            else:
                c = min(max(ps, lo), hi)
            cuts.append(c)
        bounds = [0] + cuts + [m]
        for j in range(1, len(bounds)):      # splitters are sorted, cuts must be too
            bounds[j] = max(bounds[j], bounds[j - 1])
        send = [bounds[j + 1] - bounds[j] for j in range(self.G)]
        outs, _ = self._alltoallv([keys] + payloads, send)
        keys, payloads = outs[0], outs[1:]
        keys, perm = self.ops.argsort(keys, bits)
        payloads = [self.ops.gather(p, perm) for p in payloads]
        sizes = self._gather(torch.tensor([keys.numel()], dtype=I64, device=dev)).reshape(-1).tolist()
        off = sum(sizes[: self.r])
        return keys, payloads, off, sizes

    # -- segment helpers --------------------------------------------------------
    def _neighbours(self, cols: List[torch.Tensor], m: int, dev):
        """Values of `cols` at the last element of the nearest non-empty
        previous rank and the first element of the nearest non-empty next
        rank (None when there is none)."""
        k = len(cols)
        info = torch.zeros(1 + 2 * k, dtype=I64, device=dev)
        info[0] = m
        if m:
            for j, c in enumerate(cols):
                info[1 + j] = c[0]
                info[1 + k + j] = c[-1]
        allinfo = self._gather(info).cpu().tolist()
        prev = nxt = None
        for q in range(self.r - 1, -1, -1):
            if allinfo[q][0]:
                prev = allinfo[q][1 + k: 1 + 2 * k]
                break
        for q in range(self.r + 1, self.G):
            if allinfo[q][0]:
                nxt = allinfo[q][1: 1 + k]
                break
        return prev, nxt

    def _run_flags(self, cols: List[torch.Tensor], dev):
        """head[s]: element s starts a run of equal cols; single[s]: the run
        has one element (runs may span ranks)."""
        m = cols[0].numel()
        prev, nxt = self._neighbours(cols, m, dev)
        if m == 0:
            e = torch.zeros(0, dtype=torch.bool, device=dev)
            return e, e
        diff = torch.zeros(m - 1, dtype=torch.bool, device=dev)
        for c in cols:
            diff |= c[1:] != c[:-1]
        first = prev is None or any(int(c[0]) != p for c, p in zip(cols, prev))
        last = nxt is None or any(int(c[-1]) != q for c, q in zip(cols, nxt))
        head = torch.cat([torch.tensor([first], device=dev), diff])
        nhead = torch.cat([diff, torch.tensor([last], device=dev)])
        return head, head & nhead

    def _carry_start(self, head: torch.Tensor, idx: torch.Tensor, dev) -> torch.Tensor:
        """For each element the value of idx at the last head at or before it
        (scanning across ranks): the HIP running max of idx at the heads (-1
        elsewhere); its last element, the largest head idx of this rank, is
        its carry for the next ranks."""
        m = head.numel()
        v = None
        local_last = -1
        if m:
            v = self.ops.running_max(chunked_map(lambda hd, ix: torch.where(hd, ix, -1), head, idx))
            local_last = int(v[-1].item())
        lasts = self._gather(torch.tensor([local_last], dtype=I64, device=dev)).reshape(-1).tolist()
        carry = max([-1] + lasts[: self.r])
        if m == 0:
            return idx
        return chunked_map(lambda x: torch.where(x < 0, carry, x), v)

    # -- the build ----------------------------------------------------------------
    def build(self, text: torch.Tensor, n: int) -> torch.Tensor:
        """SA[lo:hi] of this rank (int64), lo/hi = r n / G, (r+1) n / G."""
        G, r = self.G, self.r
        dev = text.device
        bnd = [n * q // G for q in range(G + 1)]
        lo, hi = bnd[r], bnd[r + 1]
        bnd_t = torch.tensor(bnd[1:-1], dtype=I64, device=dev)

        def owner(x):   # the rank whose position range holds x: boundaries <= x
            return self.ops.count_below(bnd_t, x, right=True)

        # alphabet: OR of the ranks' presence masks (torch's NCCL backend has
        # no BOR reduction, so gather the 8 words and OR them here)
        pres = torch.tensor(self.ops.alphabet(text), dtype=I64, device=dev)
        words = [0] * 8
        for row in self._gather(pres).tolist():
            words = [x | y for x, y in zip(words, row)]
        codes, sigma = [], 0
        for b in range(256):
            if (words[b >> 5] >> (b & 31)) & 1:
                sigma += 1
                codes.append(sigma)
            else:
                codes.append(0)
        K, base = choose_chars(max(sigma, 1), n)
        bits1 = bit_width(base ** K - 1)
        self.stats = {"K": K, "sigma": sigma, "rounds": 0, "distinct": [], "unsorted": []}

        # round 1: global sort of the packed K-prefixes
        keys = self.ops.pack_keys(text, n, lo, hi, codes, base, K)
        idx = torch.arange(lo, hi, dtype=I64, device=dev)
        keys, (idx,), off, _ = self._dist_sort(keys, [idx], bits1)
        m = keys.numel()
        gpos = off + torch.arange(m, dtype=I64, device=dev)
        head, single = self._run_flags([keys], dev)
        hpos = self._carry_start(head, gpos, dev)
        rank_local = torch.zeros(hi - lo, dtype=I64, device=dev)
        (ri, rv), _, _, _ = self._route(owner(idx), [idx, hpos + 1])
        self.ops.scatter(rank_local, ri, lo, rv)
        sel = self.ops.select(single)
        fin_pos, fin_idx = [self.ops.gather(gpos, sel)], [self.ops.gather(idx, sel)]
        keep = ~single
        sel = self.ops.select(keep)
        upos, uidx, uhead = (self.ops.gather(t, sel) for t in (gpos, idx, hpos))
        D = self._sum(self.ops.count_true(head), dev)
        self.stats["rounds"] = 1
        self.stats["distinct"].append(D)
        wr = bit_width(n)
        h = K
        while True:
            total_u = self._sum(uidx.numel(), dev)
            self.stats["unsorted"].append(total_u)
            if total_u == 0:
                break
            if h >= 2 * n:
                raise RuntimeError("distributed doubling did not converge")
            # rank[i + h] from its owner
            q = uidx + h
            valid = q < n
            r1 = torch.zeros_like(uidx)
            vsel = self.ops.select(valid)
            qv = self.ops.gather(q, vsel)
            (rq,), recv, order, send = self._route(owner(qv), [qv])
            (ans,), _ = self._alltoallv([self.ops.gather(rank_local, rq, lo)], recv)
            tmp = torch.empty_like(qv)
            self.ops.scatter(tmp, order, 0, ans)
            self.ops.scatter(r1, vsel, 0, tmp)
            # dense group id (groups are contiguous in SA order across ranks)
            ghead, _ = self._run_flags([uhead], dev)
            gcount = self.ops.count_true(ghead)
            gcounts = self._gather(torch.tensor([gcount], dtype=I64, device=dev)).reshape(-1).tolist()
            g = self.ops.cumsum(ghead) + (sum(gcounts[:r]) - 1)
            ngroups = sum(gcounts)
            wg = bit_width(max(ngroups - 1, 0))
            if wg + wr <= 63:
                key = (g << wr) | r1
                key, (uidx, uhead, g, r1), uoff, _ = self._dist_sort(key, [uidx, uhead, g, r1], wg + wr)
            else:   # two stable passes: by rank[i+h], then by group
                r1, (uidx, uhead, g), _, _ = self._dist_sort(r1, [uidx, uhead, g], wr)
                g, (uidx, uhead, r1), uoff, _ = self._dist_sort(g, [uidx, uhead, r1], max(wg, 1))
            mu = uidx.numel()
            uindex = uoff + torch.arange(mu, dtype=I64, device=dev)
            gstart_flag, _ = self._run_flags([g], dev)
            gstart = self._carry_start(gstart_flag, uindex, dev)
            rhead, rsingle = self._run_flags([g, r1], dev)
            rstart = self._carry_start(rhead, uindex, dev)
            pos = uhead + (uindex - gstart)
            newhead = uhead + (rstart - gstart)
            (ri, rv), _, _, _ = self._route(owner(uidx), [uidx, newhead + 1])
            self.ops.scatter(rank_local, ri, lo, rv)
            sel = self.ops.select(rsingle)
            fin_pos.append(self.ops.gather(pos, sel))
            fin_idx.append(self.ops.gather(uidx, sel))
            keep = ~rsingle
            D = (n - total_u) + self._sum(self.ops.count_true(rhead), dev)
            self.stats["rounds"] += 1
            self.stats["distinct"].append(D)
            sel = self.ops.select(keep)
            upos, uidx, uhead = (self.ops.gather(t, sel) for t in (pos, uidx, newhead))
            h *= 2
        fp = torch.cat(fin_pos)
        fi = torch.cat(fin_idx)
        (sp, si), _, _, _ = self._route(owner(fp), [fp, fi])
        sa = torch.full((hi - lo,), -1, dtype=I64, device=dev)
        self.ops.scatter(sa, sp, lo, si)
        return sa


