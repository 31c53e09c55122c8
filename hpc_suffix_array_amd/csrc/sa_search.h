// sa_search.h -- the sampled lower bound of the sparse rank look-ups
// (sa_kernels.h RankLookup::sparse, sa_dist.h), host- and device-compilable
// so that tests/test_search.py can check it against std::lower_bound with g++.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#define SA_HD __host__ __device__ __forceinline__
#else
#define SA_HD inline
#endif

namespace sa {

// Lower bound of x among the sorted key1 of SA positions [lo, hi) when the
// first round kept only every 2^ksh-th of them (keys[t] = key1 at position
// t << ksh, store_window in sa_bucket.h): an interpolation-guided search of
// the samples inside [lo, hi) narrows it to at most 2^ksh slots, searched by
// key1 rebuilt from the text at sa[p] (key_at).  ksh = 0: keys holds every
// key1.
template <class KeyAt>
SA_HD uint64_t lower_bound_sampled(const uint64_t* __restrict__ keys, uint32_t ksh,
                                                        const uint32_t* __restrict__ sa, uint64_t lo, uint64_t hi,
                                                        uint64_t x, const KeyAt& key_at) {
    if (ksh == 0) {
        uint64_t len = hi - lo;
        while (len > 0) {
            const uint64_t half = len >> 1;
            if (keys[lo + half] < x) {
                lo += half + 1;
                len -= half + 1;
            } else {
                len = half;
            }
        }
        return lo;
    }
    const uint64_t s0 = (lo + (1ull << ksh) - 1) >> ksh, s1 = (hi + (1ull << ksh) - 1) >> ksh;
    // first sample in [s0, s1) with key >= x.  The keys of one bucket are
    // near-uniform on random text, so the search starts at the position
    // interpolated between the range's end samples and gallops from there
    // (2-4 dependent loads instead of the ~9 of a binary search over ~512
    // samples); any key distribution ends in a binary search of the bracket.
    uint64_t t, len;
    {
        uint64_t a = s0, b = s1;   // answer in [a, b]
        if (s1 - s0 > 4) {
            const uint64_t klo = keys[s0], khi = keys[s1 - 1];
            if (x <= klo) {
                b = s0;
            } else if (x > khi) {
                a = s1;
            } else {
                // keys[s0] < x <= keys[s1 - 1]: guess inside (s0, s1 - 1]
                const double f = (double)(x - klo) / (double)(khi - klo);
                uint64_t g = s0 + 1 + (uint64_t)(f * (double)(s1 - 2 - s0));
                g = g < s1 - 1 ? g : s1 - 1;
                a = s0 + 1;
                b = s1 - 1;
                // gallop from g: widen until the bracket holds the answer
                uint64_t step = 1;
                if (keys[g] < x) {   // answer in (g, b]
                    uint64_t p = g;
                    for (;;) {
                        const uint64_t q = p + step < b ? p + step : b;
                        if (keys[q] >= x) {
                            a = p + 1;
                            b = q;
                            break;
                        }
                        if (q == b) {   // keys[b] >= x holds (b = s1 - 1)
                            a = b;
                            break;
                        }
                        p = q;
                        step <<= 1;
                    }
                } else {             // answer in [a, g]
                    uint64_t p = g;
                    for (;;) {
                        const uint64_t q = p >= a + step ? p - step : a;
                        if (q == a || keys[q] < x) {
                            a = q == a && !(keys[q] < x) ? a : q + 1;
                            b = p;
                            break;
                        }
                        p = q;
                        step <<= 1;
                    }
                }
            }
        }
        t = a;
        len = b - a;
        while (len > 0) {   // first t in [a, b) with keys[t] >= x, else b
            const uint64_t half = len >> 1;
            if (keys[t + half] < x) {
                t += half + 1;
                len -= half + 1;
            } else {
                len = half;
            }
        }
    }
    uint64_t l = t > s0 ? ((t - 1) << ksh) + 1 : lo;   // sample t - 1 is < x
    const uint64_t r = t < s1 ? (t << ksh) : hi;       // sample t is >= x
    // the last <= 2^ksh slots by key1 rebuilt from the text, binary (4-ary
    // steps, three rebuilds in flight per step, were slower: sort_u 0.53 ms
    // with them, 0.43 without; profiles/r03_w_ab_search.txt)
    len = r - l;
    while (len > 0) {
        const uint64_t half = len >> 1;
        if (key_at(sa[l + half]) < x) {
            l += half + 1;
            len -= half + 1;
        } else {
            len = half;
        }
    }
    return l;
}

// Every 2^ksh-th SA position inside [a + lo, a + hi) (the key samples a
// window's sub-bucket writes, sa_bucket.h k_bucket_sort): f(q) with q
// window-relative.  The first sample is found in 64 bits (a + hi reaches 2^32
// when n = 2^32); the steps stay 32-bit and window-relative, where q < hi
// (a window's size) cannot wrap.  Host-checked at the 2^32 boundary by
// tests/cpp/search_check.cpp.
template <class F>
SA_HD void for_each_sample(uint64_t a, uint32_t lo, uint32_t hi, uint32_t ksh, const F& f) {
    const uint64_t smask = (1ull << ksh) - 1ull;
    const uint64_t p0 = ((a + lo + smask) >> ksh) << ksh;
    for (uint32_t q = (uint32_t)(p0 - a); q < hi; q += (uint32_t)smask + 1u) f(q);
}

}  // namespace sa
