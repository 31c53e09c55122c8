"""Diagnostic (GPU box): the distributed driver's round-1 steps at world size 1
checked one by one at a given n (python scripts/diag_dist.py [n])."""
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from hpc_suffix_array_amd import distributed as D  # noqa: E402
from hpc_suffix_array_amd.distributed import DistributedSA, HipOps, bit_width, choose_chars  # noqa: E402


def say(*a):
    print(f"[{time.strftime('%H:%M:%S')}]", *a, flush=True)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 30
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    ops = HipOps(2 * n, 0)
    dev = ops.dev
    text = torch.empty(n, dtype=torch.uint8, device=dev)
    ops.b.generate_text(text, n, b"ACGT", seed=1, stream=torch.cuda.current_stream(dev).cuda_stream)
    codes = [0] * 256
    for j, ch in enumerate(b"ACGT"):
        codes[ch] = j + 1
    K, base = choose_chars(4, n)
    bits1 = bit_width(base ** K - 1)
    say("K", K, "bits", bits1)
    keys = ops.pack_keys(text, n, 0, n, codes, base, K)
    # spot check of the packing against the text on the host
    t_host = text[:64].cpu().tolist()
    want = 0
    for t in range(K):
        want = want * base + codes[t_host[t]]
    say("key[0]", int(keys[0]), "want", want)
    ks, perm = ops.argsort(keys, bits1)
    bad_order = int((ks[1:] < ks[:-1]).sum())
    say("sorted violations", bad_order)
    chk = ops.gather(keys, perm)
    say("gathered keys equal sorted keys", bool(torch.equal(chk, ks)))
    ps, _ = ops.argsort(perm, bit_width(n))
    say("perm is a permutation", bool(torch.equal(ps, torch.arange(n, dtype=torch.int64, device=dev))))
    d = DistributedSA(ops)
    head, single = d._run_flags([ks], dev)
    say("heads", int(head.sum()), "singles", int(single.sum()))
    keep = ~single
    sel = ops.select(keep)
    say("unsorted", sel.numel())
    gpos = torch.arange(n, dtype=torch.int64, device=dev)
    hpos = d._carry_start(head, gpos, dev)
    hp_host = hpos[:: (n // 4096) or 1]
    say("hpos monotone", bool((hpos[1:] >= hpos[:-1]).all()), "sample", hp_host[:4].tolist())
    for m in [int(x) for x in os.environ.get("DIAG_SIZES", "").split(",") if x] + [n]:
        d = DistributedSA(ops)
        try:
            sa = d.build(text[:m], m)
            say("build", m, "ok", d.stats["rounds"], d.stats["distinct"][:4], d.stats["unsorted"][:4],
                "sa head", sa[:3].tolist())
        except RuntimeError as e:
            say("build", m, "FAILED", e, d.stats["distinct"][:4], d.stats["unsorted"][:4])
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
