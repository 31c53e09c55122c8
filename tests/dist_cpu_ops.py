"""CPU stand-in for HipOps (TEST INFRASTRUCTURE ONLY): lets the distributed
driver (hpc_suffix_array_amd/distributed.py) run under gloo on CPU so its
exchange logic is tested without a GPU.  Mirrors the three local operations
of libsa_hip the driver calls: sa_alphabet_device, sa_pack_keys_device,
sa_sort_pairs_device (stable sort by key), sa_scatter_u64_device,
sa_gather_u64_device, sa_running_max_i64_device, sa_inclusive_sum_i64_device,
sa_count_below_u64_device and sa_select_u8_device."""
import torch

I64 = torch.int64


class CpuOps:
    def alphabet(self, text: torch.Tensor):
        present = torch.bincount(text.to(I64), minlength=256) > 0
        words = []
        for w in range(8):
            v = 0
            for b in range(32):
                if bool(present[32 * w + b]):
                    v |= 1 << b
            words.append(v)
        return words

    def pack_keys(self, text, n, lo, hi, codes, base, K):
        code = torch.tensor(codes, dtype=I64)[text.to(I64)]
        code = torch.cat([code, torch.zeros(K, dtype=I64)])
        x = torch.zeros(hi - lo, dtype=I64)
        for t in range(K):
            x = x * base + code[lo + t: hi + t]
        return x

    def argsort(self, keys, bits):
        ks, perm = torch.sort(keys, stable=True)
        return ks, perm

    def scatter(self, dst, idx, base, src):
        j = idx - base
        assert bool(((j >= 0) & (j < dst.numel())).all())
        dst[j] = src

    def gather(self, src, idx, base=0):
        j = idx - base
        assert bool(((j >= 0) & (j < src.numel())).all())
        return src[j]

    def running_max(self, v):
        return torch.cummax(v, 0)[0] if v.numel() else v.clone()

    def count_below(self, sorted_x, q, right=False):
        return torch.searchsorted(sorted_x, q, right=right)

    def cumsum(self, x):
        return torch.cumsum(x.to(I64), 0)

    def select(self, mask):
        return mask.nonzero().squeeze(1)

    def count_true(self, mask):
        return int(mask.sum())


class CpuRangeOps:
    """CPU stand-in for HipRangeOps (TEST INFRASTRUCTURE ONLY): the sa_dist_*
    phases of libsa_hip (csrc/sa_dist.h) restated with numpy so the
    range-partitioned driver's collectives run under gloo.  Same contracts:
    a monotone bucket of the first S symbols cut into coarse bins, identical
    cuts on every rank, round 1 = the range's suffixes sorted by their first
    K symbols, rank look-ups answered by the bucket owner (member map, else
    the round-1 group head), refinement by (group, rank[x + h])."""

    S = 2          # symbols of the bucket
    K = 3          # symbols of the first round (small: forces later rounds)

    def alphabet(self, text_slice):
        return CpuOps().alphabet(text_slice)

    def fallback_ops(self):
        return CpuOps()

    def empty(self, m, dtype):
        return torch.empty(m, dtype=dtype)

    # keys: K symbols, dense codes 1..sigma, 0 past the end, base sigma + 1
    def _keys(self, pos, K):
        import numpy as np
        x = np.zeros(len(pos), dtype=np.int64)
        for t in range(K):
            q = pos + t
            c = np.where(q < self.n, self.code[np.minimum(q, self.n - 1)], 0)
            x = x * self.base + c
        return x

    def _coarse(self, pos):
        import numpy as np
        ks = self._keys(pos, self.S)
        return (ks * 4096 // (self.base ** self.S)).astype(np.int64)

    def begin(self, text, n, world, rank, present):
        import numpy as np
        self.t = text.numpy().astype(np.int64)
        self.n, self.G, self.r = n, world, rank
        code = np.zeros(256, dtype=np.int64)
        sigma = 0
        for b in range(256):
            if (present[b >> 5] >> (b & 31)) & 1:
                sigma += 1
                code[b] = sigma
        self.code = code[self.t]
        self.sigma, self.base = sigma, sigma + 1
        info = {"status": 0 if sigma >= 2 else 1, "sigma": sigma, "K": self.K, "bucket_bits": 12}
        lo, hi = n * rank // world, n * (rank + 1) // world
        hist = np.bincount(self._coarse(np.arange(lo, hi)), minlength=4096) if sigma >= 2 else np.zeros(4096)
        return info, torch.from_numpy(hist.astype(np.int64))

    def cuts(self, coarse_host):
        import numpy as np
        G, n = self.G, self.n
        h = np.bincount(self._coarse(np.arange(n)), minlength=4096) if coarse_host is None else coarse_host.numpy()
        pre = np.concatenate([[0], np.cumsum(h)])
        cut = [0] * (G + 1)
        cut[G] = 4096
        for q in range(1, G):
            cut[q] = int(np.searchsorted(pre, n * q // G, side="left"))
            cut[q] = max(cut[q], cut[q - 1])
        self.cut = cut
        self.owner_tab = np.zeros(4096, dtype=np.int64)
        for q in range(G):
            self.owner_tab[cut[q]:cut[q + 1]] = q
        self.m = int(pre[cut[self.r + 1]] - pre[cut[self.r]])
        self.sa_off = int(pre[cut[self.r]])
        mmax = max(int(pre[cut[q + 1]] - pre[cut[q]]) for q in range(G))
        ok = mmax <= n // G + n // G // 2 + 65536
        return {"status": 0 if ok else 2, "m": self.m, "sa_off": self.sa_off, "m_max": mmax}

    def round1(self, sa_local):
        import numpy as np
        pos = np.arange(self.n)
        mine = pos[(self._coarse(pos) >= self.cut[self.r]) & (self._coarse(pos) < self.cut[self.r + 1])]
        k = self._keys(mine, self.K)
        o = np.lexsort((mine, k))
        sa = mine[o]
        self.keys1 = k[o]
        sa_local[:] = torch.from_numpy(sa.astype(np.int64)).to(sa_local.dtype)
        self.grank = {}
        self._set_u(self.keys1, sa, np.arange(len(sa)), first=True)
        return {"round1_ok": 1, "heads": self.heads, "unsorted": len(self.u_idx), "groups": self.gu}

    def _set_u(self, keys, idx, positions, first=False):
        """groups of equal keys (sorted order) -> heads, ranks, next unsorted set"""
        import numpy as np
        m = len(keys)
        head = np.ones(m, dtype=bool)
        if m > 1:
            head[1:] = keys[1:] != keys[:-1]
        nxt = np.ones(m, dtype=bool)
        if m > 1:
            nxt[:-1] = head[1:]
        single = head & nxt
        run_start = np.maximum.accumulate(np.where(head, np.arange(m), 0)) if m else np.zeros(0, np.int64)
        self.heads = int(head.sum())
        inu = ~single
        for s_ in np.nonzero(inu if first else np.ones(m, dtype=bool))[0]:
            self.grank[int(idx[s_])] = self.sa_off + int(positions[run_start[s_]]) + 1
        g = np.cumsum(head & inu) - 1
        self.u_pos = positions[inu]
        self.u_idx = idx[inu]
        self.u_g = g[inu]
        self.gu = int((head & inu).sum())

    def req_count(self, h, world):
        import numpy as np
        j = self.u_idx + h
        ok = j < self.n
        self.req_owner = np.full(len(j), -1)
        if ok.any():
            self.req_owner[ok] = self.owner_tab[self._coarse(j[ok])]
        counts = [int((self.req_owner == q).sum()) for q in range(world)]
        return counts, {"unsorted": len(self.u_idx), "groups": self.gu}

    def req_fill(self, h, nsend):
        import numpy as np
        sel = np.nonzero(self.req_owner >= 0)[0]
        o = sel[np.argsort(self.req_owner[sel], kind="stable")]
        self.perm = o
        assert len(o) == nsend
        return torch.from_numpy((self.u_idx[o] + h).astype(np.int64)).to(torch.int32)

    def answer(self, req):
        import numpy as np
        j = req.numpy().astype(np.int64) & 0xFFFFFFFF
        out = np.zeros(len(j), dtype=np.int64)
        if len(j):
            c = self._coarse(j)
            assert ((c >= self.cut[self.r]) & (c < self.cut[self.r + 1])).all(), "request outside the range"
            kj = self._keys(j, self.K)
            lo = np.searchsorted(self.keys1, kj, side="left")
            for t in range(len(j)):
                out[t] = self.grank.get(int(j[t]), self.sa_off + int(lo[t]) + 1)
        return torch.from_numpy(out)

    def refine(self, h, ans, sa_local):
        import numpy as np
        m = len(self.u_idx)
        if m == 0:
            return {"heads": 0, "unsorted": 0, "groups": 0}
        r1 = np.zeros(m, dtype=np.int64)
        r1[self.perm] = ans.numpy()
        o = np.lexsort((r1, self.u_g))
        idx, g, r = self.u_idx[o], self.u_g[o], r1[o]
        positions = self.u_pos   # sorted index s -> SA position u_pos[s] (groups keep their ranges)
        sa_local[torch.from_numpy(positions.astype(np.int64))] = torch.from_numpy(idx.astype(np.int64)).to(
            sa_local.dtype)
        key = g.astype(object) * (self.n + 2) + r.astype(object)
        key = np.array([int(x) for x in key], dtype=object)
        keys = np.zeros(m, dtype=np.int64)
        keys[0] = 0
        if m > 1:
            keys[1:] = np.cumsum(key[1:] != key[:-1])
        self._set_u(keys, idx, positions)
        return {"heads": self.heads, "unsorted": len(self.u_idx), "groups": self.gu}
