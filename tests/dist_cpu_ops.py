"""CPU stand-in for HipOps (TEST INFRASTRUCTURE ONLY): lets the distributed
driver (hpc_suffix_array_amd/distributed.py) run under gloo on CPU so its
exchange logic is tested without a GPU.  Mirrors the three local operations
of libsa_hip the driver calls: sa_alphabet_device, sa_pack_keys_device,
sa_sort_pairs_device (stable sort by key), sa_scatter_u64_device, sa_gather_u64_device, sa_running_max_i64_device."""
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
