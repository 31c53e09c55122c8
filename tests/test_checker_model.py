"""The permutation checker's formulation (hpc_suffix_array_amd/csrc/sa_check.h),
restated in numpy, against the oracle's direct check of every adjacent pair
(oracle/mm_oracle.c, manber_myers.c:184-202).

sa_check.h does not compare SA[r-1] and SA[r] through random gathers: pass A
places ISA'[SA[r]] = r + 1 (and proves SA a permutation by exact bin counts,
no holes), pass B places at r = ISA[i] the key (text[i] << 32 | ISA'[i+1])
(ISA'[n] = 0) and checks that the keys rise strictly along r.  This file
checks that the two verdicts agree on valid suffix arrays and on every kind of
corruption (host only; the kernels themselves are tested on the GPU by
tests/test_gpu_parity.py::test_checker_permutation_passes)."""
import numpy as np
import pytest


def check_model(text: np.ndarray, sa: np.ndarray) -> bool:
    n = len(text)
    sa = sa.astype(np.int64)
    if n == 0:
        return True
    if (sa < 0).any() or (sa >= n).any():
        return False
    isa1 = np.zeros(n, np.int64)             # pass A: ISA' = r + 1, 0 = hole
    isa1[sa] = np.arange(1, n + 1)
    if (isa1 == 0).any() or len(np.unique(sa)) != n:
        return False
    nxt = np.zeros(n, np.int64)
    nxt[:-1] = isa1[1:]                        # ISA'[i + 1], ISA'[n] = 0
    keys = np.empty(n, np.int64)               # pass B: key placed at ISA[i]
    keys[isa1 - 1] = (text.astype(np.int64) << 32) | nxt
    return bool((keys[1:] > keys[:-1]).all())


@pytest.mark.parametrize("kind", ["dna", "alnum", "binary", "byte256"])
@pytest.mark.parametrize("n", [1, 2, 3, 17, 1000, 40_000])
def test_model_agrees_with_oracle(oracle, kind, n):
    rng = np.random.default_rng(n * 7 + len(kind))
    t = oracle.gen_text(kind, n, seed=n)
    sa = oracle.sa_c(t)
    assert check_model(t, sa) and oracle.check_c(t, sa)
    variants = [sa[::-1].copy(), np.arange(n, dtype=sa.dtype)]
    for _ in range(20):
        v = sa.copy()
        i, j = rng.integers(0, n, 2)
        op = rng.integers(0, 3)
        if op == 0:
            v[[i, j]] = v[[j, i]]
        elif op == 1:
            v[i] = v[j]
        else:
            k = int(rng.integers(0, max(1, n - 8)))
            v[k:k + 8] = rng.permutation(v[k:k + 8])
        variants.append(v)
    for v in variants:
        assert check_model(t, v) == oracle.check_c(t, v)


def test_model_runs_and_degenerate(oracle):
    for t in (np.full(5000, ord("a"), np.uint8), np.tile(np.frombuffer(b"abaab", np.uint8), 999)):
        sa = oracle.sa_c(t)
        assert check_model(t, sa)
        bad = sa.copy()
        bad[[0, -1]] = bad[[-1, 0]]
        assert not check_model(t, bad)
