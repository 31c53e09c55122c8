// g++ host check of sa_limits.h (tests/test_limits.py): the per-XCD second
// pass is gated off exactly where its 32-bit region offsets would wrap.
#include <cstdio>

#include "../../hpc_suffix_array_amd/csrc/sa_limits.h"

int main() {
    using namespace sa;
    int bad = 0;
    // the largest m whose regions fit: m + m/16 + 8*1024*2048 <= 2^32 - 1
    uint64_t lo = 0, hi = 1ull << 33;
    while (lo + 1 < hi) {
        const uint64_t mid = (lo + hi) / 2;
        (xq_offsets_fit(mid) ? lo : hi) = mid;
    }
    const uint64_t mmax = lo;
    bad += !(xq_region_space(mmax) <= 0xFFFFFFFFull);
    bad += !(xq_region_space(mmax + 1) > 0xFFFFFFFFull);
    bad += xq_offsets_fit(mmax + 1);
    // one GPU: every n up to 2^31 (the bucketed round's maximum) keeps XQ;
    // a single device's 2^32 - 1 does not
    bad += !xq_offsets_fit(1ull << 31);
    bad += xq_offsets_fit(0xFFFFFFFFull);
    bad += !(mmax > 3900000000ull && mmax < 4100000000ull);
    std::printf("xq max m %llu bad %d\n", (unsigned long long)mmax, bad);
    return bad ? 1 : 0;
}
