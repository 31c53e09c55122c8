"""CPU check of the bucketed first round's key layout (sa_bucket.h, the
BucketSpec/key1_at of sa_kernels.h), restated in Python: key1 must order
suffixes exactly as their first K = s + R symbols with the end of the text
smallest (manber_myers.c:91,122 sentinel), give equal keys exactly to equal
K-prefixes, and its 16-bit bucket must be monotone in key1.  Both fields
are dense (digits code - 1, the end clamped onto the smallest symbol's
digit), and the count of symbols before the end separates the suffixes that
the clamp merges.  Small alphabets
and small s make every corner (suffixes shorter than s, shorter than K)
common.  The compact variant (BucketSpec.cmp: low = 2 r + [L >= K] for every suffix)
is checked on every text for which the host's precondition
(short_suffix_ties, sa_round1.h) lets it be chosen, and the precondition is
checked to be necessary."""
import itertools
import random

import pytest


def key1(text, i, sigma, s, R, code, cmp=False):
    n = len(text)
    D = 0
    for t in range(s):
        c = code[text[i + t]] if i + t < n else 0
        D = D * sigma + (c - 1 if c else 0)
    L = n - i
    r = 0
    for t in range(R):
        c = code[text[i + s + t]] if i + s + t < n else 0
        r = r * sigma + (c - 1 if c else 0)
    if cmp:
        low = 2 * r + (1 if L >= s + R else 0)
    elif L < s:
        low = L - 1
    else:
        low = s + r * (R + 1) + min(R, L - s)
    rb = (2 * sigma ** R - 1 if cmp else s + (sigma ** R - 1) * (R + 1) + R).bit_length()
    return (D << rb) | low, rb


def short_suffix_ties(text, sigma, s, R, code):
    """sa_round1.h short_suffix_ties: two of the last K - 1 suffixes with
    equal (D, r) (digits 0 past the end)."""
    n, K = len(text), s + R
    seen = set()
    for L in range(1, min(K, n + 1)):
        i = n - L
        dr = tuple((code[text[i + t]] - 1) if i + t < n else 0 for t in range(K))
        if dr in seen:
            return True
        seen.add(dr)
    return False


def prefix(text, i, K):
    # K-prefix with the end smallest: symbols shifted by one, 0 past the end
    return tuple((text[i + t] + 1) if i + t < len(text) else 0 for t in range(K))


@pytest.mark.parametrize("sigma,s,R", [(2, 3, 2), (2, 1, 4), (3, 2, 2), (4, 3, 1), (5, 2, 3), (2, 2, 5)])
def test_key1_orders_like_k_prefix(sigma, s, R):
    rng = random.Random(sigma * 100 + s * 10 + R)
    code = {b: b + 1 for b in range(sigma)}   # dense codes 1..sigma
    K = s + R
    for _ in range(60):
        n = rng.randint(1, 14)
        text = [rng.randrange(sigma) for _ in range(n)]
        if rng.random() < 0.3:
            text = [0] * n   # runs of the smallest symbol collide with shorter suffixes under the clamp
        keys = [key1(text, i, sigma, s, R, code)[0] for i in range(n)]
        pre = [prefix(text, i, K) for i in range(n)]
        for a, b in itertools.combinations(range(n), 2):
            assert (keys[a] < keys[b]) == (pre[a] < pre[b]), (text, a, b)
            assert (keys[a] == keys[b]) == (pre[a] == pre[b]), (text, a, b)


@pytest.mark.parametrize("sigma,s,R", [(2, 3, 2), (2, 1, 4), (3, 2, 2), (4, 3, 1), (5, 2, 3), (2, 2, 5), (4, 2, 4)])
def test_compact_key1_orders_like_k_prefix(sigma, s, R):
    rng = random.Random(sigma * 1000 + s * 10 + R)
    code = {b: b + 1 for b in range(sigma)}
    K = s + R
    used = ties = 0
    for _ in range(300):
        n = rng.randint(1, 16)
        text = [rng.randrange(sigma) for _ in range(n)]
        if rng.random() < 0.3:   # runs of the smallest symbol at the end
            text[rng.randrange(n):] = [0] * (n - rng.randrange(n)) if n else []
            text = text[:n] + [0] * (n - len(text))
        keys = [key1(text, i, sigma, s, R, code, cmp=True)[0] for i in range(n)]
        pre = [prefix(text, i, K) for i in range(n)]
        ok = all((keys[a] < keys[b]) == (pre[a] < pre[b]) and (keys[a] == keys[b]) == (pre[a] == pre[b])
                 for a, b in itertools.combinations(range(n), 2))
        if short_suffix_ties(text, sigma, s, R, code):
            ties += 1
        else:
            used += 1
            assert ok, (text, keys)
    assert used > 100
    if R >= 2 and s <= 2:
        assert ties > 0   # the precondition does reject some texts here


def test_compact_precondition_is_necessary():
    # DNA-like: the text ends in a run of the smallest symbol, so its last
    # suffixes "A", "AA", ... pad to the same (D, r)
    sigma, s, R = 4, 2, 3
    code = {b: b + 1 for b in range(sigma)}
    text = [1, 2, 3, 0, 0, 0, 0, 0]
    assert short_suffix_ties(text, sigma, s, R, code)
    keys = [key1(text, i, sigma, s, R, code, cmp=True)[0] for i in range(len(text))]
    pre = [prefix(text, i, s + R) for i in range(len(text))]
    assert any(keys[a] == keys[b] and pre[a] != pre[b] for a, b in itertools.combinations(range(len(text)), 2))


def test_bucket_monotone():
    # bucket = (D * cmul) >> 32 with cmul = floor(2^48 / sigma^s) < 2^16
    for sigma in (2, 3, 4, 62, 127, 256):
        ps, s = 1, 0
        while ps < 65536:
            ps *= sigma
            s += 1
        cmul = (1 << 48) // ps
        prev = -1
        for D in list(range(0, min(ps, 5000))) + list(range(max(0, ps - 5000), ps)):
            b = (D * cmul) >> 32
            assert 0 <= b < 65536 and b >= prev
            prev = b
        assert (((ps - 1) * cmul) >> 32) > 65000   # the 16 bits are used
