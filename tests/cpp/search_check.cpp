// Host check of sa::lower_bound_sampled (hpc_suffix_array_amd/csrc/sa_search.h)
// against std::lower_bound: sorted keys with uniform, clustered, duplicated
// and two-valued distributions, every 2^ksh-th key kept as a sample (ksh 0 and
// 4, as the bucketed first round keeps them), random [lo, hi) ranges and
// probes inside, between and outside the keys.  Prints "ok <cases>" or the
// first mismatch.  Built by tests/test_search.py with g++.
#include <algorithm>
#include <cstdio>
#include <cmath>
#include <random>
#include <vector>

#include "sa_search.h"

int main() {
    std::mt19937_64 rng(12345);
    long cases = 0;
    for (int dist = 0; dist < 5; ++dist) {
        for (uint32_t ksh : {0u, 4u}) {
            for (int rep = 0; rep < 40; ++rep) {
                const uint64_t n = 1 + rng() % 20000;
                std::vector<uint64_t> full(n);
                for (auto& v : full) {
                    switch (dist) {
                        case 0: v = rng(); break;                                  // uniform 64-bit
                        case 1: v = rng() % 1000; break;                           // many duplicates
                        case 2: v = (rng() % 16 == 0) ? rng() : (1ull << 40); break;   // one dominant value
                        case 3: v = (rng() & 1) ? rng() % 100 : (1ull << 62) + rng() % 100; break;   // two clusters
                        default: v = (uint64_t)std::exp2((double)(rng() % 6000) / 100.0); break;   // skewed
                    }
                }
                std::sort(full.begin(), full.end());
                // samples: keys[t] = full[t << ksh]; sa[p] = p, key_at(p) = full[p]
                std::vector<uint64_t> samples((n + (1ull << ksh) - 1) >> ksh);
                for (uint64_t t = 0; t < samples.size(); ++t) samples[t] = full[t << ksh];
                std::vector<uint32_t> sa(n);
                for (uint64_t p = 0; p < n; ++p) sa[p] = (uint32_t)p;
                auto key_at = [&](uint32_t p) { return full[p]; };
                for (int q = 0; q < 200; ++q) {
                    uint64_t lo = rng() % (n + 1), hi = rng() % (n + 1);
                    if (lo > hi) std::swap(lo, hi);
                    uint64_t x;
                    const int kind = (int)(rng() % 4);
                    if (kind == 0 && hi > lo) x = full[lo + rng() % (hi - lo)];          // a key of the range
                    else if (kind == 1 && hi > lo) x = full[lo + rng() % (hi - lo)] + 1;  // just above one
                    else if (kind == 2) x = rng() % 4 ? 0 : ~0ull;                         // outside
                    else x = rng();
                    const uint64_t want = (uint64_t)(std::lower_bound(full.begin() + lo, full.begin() + hi, x) - full.begin());
                    const uint64_t got = sa::lower_bound_sampled(samples.data(), ksh, sa.data(), lo, hi, x, key_at);
                    ++cases;
                    if (got != want) {
                        std::printf("mismatch dist %d ksh %u n %llu lo %llu hi %llu x %llu: got %llu want %llu\n", dist,
                                    ksh, (unsigned long long)n, (unsigned long long)lo, (unsigned long long)hi,
                                    (unsigned long long)x, (unsigned long long)got, (unsigned long long)want);
                        return 1;
                    }
                }
            }
        }
    }
    // sa::for_each_sample (the local sort's key samples) against a 64-bit
    // scan, windows ending at and just below 2^32 (n = 2^32, world 1 or a
    // range build's last range) and random windows
    {
        auto check = [&](uint64_t a, uint32_t lo, uint32_t hi, uint32_t ksh) {
            std::vector<uint64_t> got, want;
            sa::for_each_sample(a, lo, hi, ksh, [&](uint32_t q) {
                got.push_back(a + q);
                if (got.size() > hi - lo + 1) return;
            });
            for (uint64_t p = a + lo; p < a + hi; ++p)
                if ((p & ((1ull << ksh) - 1)) == 0) want.push_back(p);
            ++cases;
            if (got != want) {
                std::printf("for_each_sample mismatch a %llu lo %u hi %u ksh %u: %zu vs %zu samples\n",
                            (unsigned long long)a, lo, hi, ksh, got.size(), want.size());
                return false;
            }
            return true;
        };
        for (uint32_t ksh : {0u, 1u, 4u}) {
            for (uint32_t w : {1u, 7u, 16u, 17u, 9216u}) {
                for (uint64_t end : {1ull << 32, (1ull << 32) - 1, (1ull << 32) - 16, (1ull << 32) + 0x1234}) {
                    for (uint32_t lo : {0u, 1u, w / 2}) {
                        if (!check(end - w, lo, w, ksh)) return 1;
                        if (lo < w && !check(end - w, lo, w - 1, ksh)) return 1;
                    }
                }
            }
            for (int rep = 0; rep < 2000; ++rep) {
                const uint32_t w = 1 + (uint32_t)(rng() % 9216);
                const uint64_t a = rng() % ((1ull << 33) - w);
                const uint32_t lo = (uint32_t)(rng() % (w + 1)), hi = lo + (uint32_t)(rng() % (w - lo + 1));
                if (!check(a, lo, hi, ksh)) return 1;
            }
        }
    }
    std::printf("ok %ld\n", cases);
    return 0;
}
