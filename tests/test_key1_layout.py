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
    if cmp == 2:     # E-only: no end bit (BucketSpec.cmp = 2)
        low = r
    elif cmp:
        low = 2 * r + (1 if L >= s + R else 0)
    elif L < s:
        low = L - 1
    else:
        low = s + r * (R + 1) + min(R, L - s)
    rb = ((sigma ** R - 1) if cmp == 2 else 2 * sigma ** R - 1 if cmp else
          s + (sigma ** R - 1) * (R + 1) + R).bit_length()
    return (D << rb) | low, rb


def short_suffix_ties(text, sigma, s, R, code, last=None):
    """sa_round1.h short_suffix_ties: two of the last K - 1 suffixes (`last`
    of them: K for the E-only layout) with equal (D, r) (digits 0 past the
    end)."""
    n, K = len(text), s + R
    last = K - 1 if last is None else last
    seen = set()
    for L in range(1, min(last + 1, n + 1)):
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


def packed_doubling(text, sigma, s, R, code, cmp):
    """The packed schedule on key1: round 1 groups the
    suffixes by key1 (groups keep their SA ranges in key1 order, rank = the
    group's first position + 1), then rounds h = K, 2K, ... sort every group
    by rank[i + h] (0 past the end) until all groups are singletons."""
    n, K = len(text), s + R
    keys = [key1(text, i, sigma, s, R, code, cmp=cmp)[0] for i in range(n)]
    sa = sorted(range(n), key=lambda i: keys[i])
    grp = [0] * n   # group id = its first SA position
    for p in range(1, n):
        grp[sa[p]] = grp[sa[p - 1]] if keys[sa[p]] == keys[sa[p - 1]] else p
    h = K
    for _ in range(64):
        rank = [g + 1 for g in grp]
        if len(set(grp)) == n:
            return sa
        sa = sorted(range(n), key=lambda i: (grp[i], rank[i + h] if i + h < n else 0))
        new = [0] * n
        for p in range(1, n):
            a, b = sa[p - 1], sa[p]
            same = grp[a] == grp[b] and (rank[a + h] if a + h < n else 0) == (rank[b + h] if b + h < n else 0)
            new[b] = new[a] if same else p
        grp = new
        h *= 2
    raise AssertionError("doubling did not converge")


@pytest.mark.parametrize("sigma,s,R", [(2, 3, 2), (2, 1, 4), (3, 2, 2), (4, 3, 1), (5, 2, 3), (2, 2, 5), (4, 2, 4)])
def test_eonly_key1_doubling_gives_the_sa(sigma, s, R):
    """The E-only layout (BucketSpec.cmp = 2: low = r, no end bit; one bit
    less than the compact layout, which lets non-power-of-two alphabets take
    packed 8-byte first-pass items): a short suffix S (length L < K) shares
    its key with the suffixes continuing it with the smallest symbol, and
    round 2 separates them (S + K is past the end: rank 0).  Exact when the
    last K suffixes (lengths 1..K) have distinct padded keys, which the host
    checks (short_suffix_ties over K): the packed doubling on it gives the
    suffix array on every such text, and its key order never contradicts the
    K-prefix order."""
    rng = random.Random(sigma * 7919 + s * 31 + R)
    code = {b: b + 1 for b in range(sigma)}
    K = s + R
    used = rejected = 0
    for _ in range(400):
        n = rng.randint(1, 18)
        text = [rng.randrange(sigma) for _ in range(n)]
        if rng.random() < 0.3:   # runs of the smallest symbol at the end
            k = rng.randrange(n + 1)
            text = text[:k] + [0] * (n - k)
        if short_suffix_ties(text, sigma, s, R, code, last=K):
            rejected += 1
            continue
        used += 1
        keys = [key1(text, i, sigma, s, R, code, cmp=2)[0] for i in range(n)]
        pre = [prefix(text, i, K) for i in range(n)]
        for a, b in itertools.combinations(range(n), 2):
            if keys[a] < keys[b]:
                assert pre[a] < pre[b], (text, a, b)
            elif keys[a] > keys[b]:
                assert pre[a] > pre[b], (text, a, b)
        want = sorted(range(n), key=lambda i: [x + 1 for x in text[i:]])
        assert packed_doubling(text, sigma, s, R, code, 2) == want, text
    assert used > 150 and rejected > 0


def test_eonly_precondition_is_needed():
    """Without the check the E-only keys can tie a short suffix with the
    length-K suffix forever: "...AAA" with K = 3 (S = "A", T = "AAA")."""
    sigma, s, R = 4, 1, 2
    code = {b: b + 1 for b in range(sigma)}
    text = [2, 1, 0, 0, 0]
    assert short_suffix_ties(text, sigma, s, R, code, last=3)
    with pytest.raises(AssertionError):
        assert packed_doubling(text, sigma, s, R, code, 2) == sorted(range(5), key=lambda i: [x + 1 for x in text[i:]])


@pytest.mark.parametrize("sigma,s,bb", [(3, 11, 16), (5, 7, 17), (62, 3, 16), (62, 5, 18), (95, 4, 18),
                                        (127, 4, 18), (200, 4, 18), (255, 4, 18), (10, 9, 17)])
def test_bucket_relative_d_from_the_fraction(sigma, s, bb):
    """k_split_text's NP2 items (sa_split.h): D - Dmin(bucket) computed as
    floor(f / cmul), f = D cmul mod 2^bsh, by a double reciprocal corrected
    one step each way, equals D - bucket_dmin(bucket) (sa_bucket.h:90) at
    every bucket edge and at random D."""
    ps = sigma ** s
    cmul = (1 << 48) // ps
    bsh = 48 - bb
    icm = 1.0 / cmul

    def dmin(b):
        d0 = (b << bsh) // cmul
        return d0 if (d0 * cmul) >> bsh == b else d0 + 1

    def rel(D):
        prod = D * cmul
        f = prod & ((1 << bsh) - 1)
        rd = int(float(f) * icm)
        if rd * cmul > f:
            rd -= 1
        if (rd + 1) * cmul <= f:
            rd += 1
        return prod >> bsh, rd

    rng = random.Random(sigma * 1009 + s)
    Ds = {0, ps - 1}
    for _ in range(3000):
        b = rng.randrange(1 << bb)
        d = dmin(b)
        Ds.update(x for x in (d - 1, d, d + 1) if 0 <= x < ps)
        Ds.add(rng.randrange(ps))
    for D in Ds:
        b, rd = rel(D)
        assert rd == D - dmin(b), (D, b)
