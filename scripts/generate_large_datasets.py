#!/usr/bin/env python3
"""Seeded stand-in for the reference's scripts/generate_large_datasets.py.

Same files and shapes (random = ascii_letters + digits, :12-14; repetitive
1000-char lowercase pattern, :16-23; DNA = ACGT, :25-28; sizes in MiB, :55-60;
small cases :90-96), but reproducible: symbols come from the splitmix64
generator of SURVEY.md 8(d) instead of unseeded random.choices.

    python scripts/generate_large_datasets.py [--sizes 1 50 ...] [--seed 1]
"""
import argparse
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ALNUM = b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789"


def splitmix_text(alphabet: bytes, n: int, seed: int) -> bytes:
    alpha = np.frombuffer(alphabet, dtype=np.uint8)
    sigma = np.uint64(len(alpha))
    out = np.empty(n, dtype=np.uint8)
    with np.errstate(over="ignore"):
        for lo in range(0, n, 1 << 24):
            hi = min(n, lo + (1 << 24))
            z = np.uint64(seed) + np.arange(lo + 1, hi + 1, dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15)
            z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
            z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
            z = z ^ (z >> np.uint64(31))
            out[lo:hi] = alpha[((z >> np.uint64(32)) * sigma) >> np.uint64(32)]
    return out.tobytes()


def save(path: str, content: bytes, description: str) -> None:
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "wb") as f:
        f.write(content)
    with open(path + ".meta", "w") as f:
        f.write(f"Description: {description}\nLength: {len(content)} characters\n")
        f.write(f"MD5: {hashlib.md5(content).hexdigest()}\n")
    print(f"Generated: {path} ({len(content):,} bytes)")


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", type=int, nargs="*", default=[1, 50, 100, 200, 500])
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default=os.path.join(ROOT, "test_data"))
    a = ap.parse_args(argv)
    for mb in a.sizes:
        n = mb * 1024 * 1024
        save(os.path.join(a.out, "large", f"random_{mb}MB.txt"), splitmix_text(ALNUM, n, a.seed),
             f"random alnum {mb} MiB")
    pattern = splitmix_text(b"abcdefghijklmnopqrstuvwxyz", 1000, a.seed + 1)
    n = 10 * 1024 * 1024
    save(os.path.join(a.out, "large", "repetitive_10MB.txt"), (pattern * (n // 1000 + 1))[:n], "repetitive")
    save(os.path.join(a.out, "large", "dna_10MB.txt"), splitmix_text(b"ACGT", n, a.seed), "DNA")
    for name, s in (("banana", b"banana"), ("mississippi", b"mississippi"), ("abcabcabc", b"abcabcabc"),
                    ("aaaa", b"a" * 1000), ("ababab", b"ab" * 500)):
        save(os.path.join(a.out, f"{name}.txt"), s, name)
    return 0


if __name__ == "__main__":
    sys.exit(main())
