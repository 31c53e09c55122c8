// sa_limits.h -- host-side size gates of the round-1 plan, kept free of HIP
// so that tests/cpp/limits_check.cpp can check them with g++ at the
// boundaries the device code cannot be driven to in a test.
#pragma once
#include <cstdint>

namespace sa {

constexpr uint32_t kXqQueues = 8;             // per-XCD queues of the second bucket pass (sa_split.h kXq)
constexpr uint32_t kXqRegionSlack = 2048;     // per (queue, digit) sub-region slack (sa_split.h kXqSlack)
constexpr uint32_t kXqMaxDigits = 1024;       // the second pass's widest digit (10 bits)

// Items of the second pass's 8 per-XCD output regions for m suffixes: digit
// h of queue q gets tot(h)/8 + tot(h)/128 + slack (k_xq_dh), so the regions
// hold at most m + m/16 + 8 * 1024 * slack items.
constexpr uint64_t xq_region_space(uint64_t m) {
    return m + m / 16 + (uint64_t)kXqQueues * kXqMaxDigits * kXqRegionSlack;
}

// The regions are addressed with 32-bit offsets (k_split_seg<.., XQ>,
// k_bucket_starts_xq, load_items_xq): the XQ pass runs only when every
// offset fits (past ~4.02e9 suffixes queue 7 wrapped onto region 0).
constexpr bool xq_offsets_fit(uint64_t m) { return xq_region_space(m) <= 0xFFFFFFFFull; }

}  // namespace sa
