// sa_pivot.h -- three-way pivot split of an unsorted-set round with large
// groups (Larsson-Sadakane's ternary split, applied once per round).
//
// An unsorted-set round (packed schedule, rounds h >= K) sorts every group g
// of the unsorted set U by its members' keys rank[x + h] (manber_myers.c:98,
// the two counting passes, restricted to U).  Ties may end in any order: the
// round only needs the classes of equal keys.  When groups are large, most
// members of a group often share one key -- a text of one repeated symbol
// (configs[4]: every round keeps one group of ~n members, all but ~h of them
// with the group's own rank as key), long repeats, short periods.  There the
// LSD sort of all m members (4 passes of 12 bytes at 2^30) moves everything
// to reorder a few.  Instead, per group, with pivot p = the key of the
// group's first member:
//   * members with key == p keep nothing but their group: they are written
//     once, in U order, as one tied block;
//   * members with key < p and key > p (the "rest", m' of them) are sorted by
//     (2 g + [key > p], key) with the ordinary radix sort and placed before /
//     after the tied block.
// New layout of group g (its U slots [gs_g, gs_{g+1}) keep their SA
// positions): [< p sorted][== p][> p sorted].  segments() then sees the same
// (key, index) stream a full sort would produce, up to the order of ties.
//
// Kernels (Chunking over U, one workgroup per chunk walking 4096-member
// tiles; wave w owns a contiguous 1024 slice, rows of 64 lanes):
//   k_pivot_keys    key(e) = g << wr | rank[x + h] (dense ranks), the
//                   group starts gs[g] (gs[G] = m) and the pivots' ranks
//                   pr[g] (the passes read a member's pivot with one
//                   dependent load, pr[g], instead of two, keys[gs[g]])
//   k_pivot_pass<0> class counts per chunk (k_scan_rows then gives P_c at
//                   each chunk start) and per group start inside its chunk
//   k_pivot_gp      gP[c][g] = P_c(gs_g) (members of class c before g)
//   k_pivot_pass<2> tied members to their final slots, the rest compacted
//   k_pivot_place   the sorted rest to their final slots
// Tied-block round (pivot_round's default when G is small): the tied block of
// group g is already one group of the next round, so nothing of it needs the
// segment scan -- k_pivot_pass<3> writes each tied member's rank (its block's
// first SA position + 1, as k_seg_write would), the SA entry of a one-member
// block, and the next unsorted set's entries (u_pos, u_idx, u_g) of blocks of
// two or more at the front of that set (block ids 0..Gt-1 in group order,
// offsets from k_pivot_tied_scan); only the sorted rest goes through
// segments(), appended after them with group ids from Gt.  Per tied member
// 28 bytes (key and u_idx read; rank and three set words written) instead
// of the 80 of pass<2> + k_seg_count + k_seg_write.  (The passes take a
// member's group from its key, g = key >> wr, not from u_g.)
#pragma once
#include <type_traits>

#include "sa_kernels.h"

namespace sa {

// keys of a pivot round (dense ranks only) and the group starts; kPkItems
// members per thread, all loads of a batch issued before the rank gathers
// that depend on them
constexpr int kPkItems = 4;
__global__ __launch_bounds__(kBlock) void k_pivot_keys(const uint32_t* __restrict__ u_idx,
                                                       const uint32_t* __restrict__ u_g, uint64_t m,
                                                       const uint32_t* __restrict__ rank, uint64_t n, uint64_t h,
                                                       uint32_t wr, uint32_t G, uint64_t* __restrict__ keys,
                                                       uint32_t* __restrict__ gs, uint32_t* __restrict__ pr) {
    const uint64_t step = (uint64_t)gridDim.x * kBlock * kPkItems;
    for (uint64_t base = (uint64_t)blockIdx.x * kBlock * kPkItems; base < m; base += step) {
        uint32_t x[kPkItems], g[kPkItems], gp[kPkItems], r1[kPkItems];
#pragma unroll
        for (int i = 0; i < kPkItems; ++i) {
            const uint64_t e = base + (uint64_t)i * kBlock + threadIdx.x;
            x[i] = e < m ? u_idx[e] : 0u;
            g[i] = e < m ? u_g[e] : 0u;
            gp[i] = (e < m && e > 0) ? u_g[e - 1] : ~0u;
        }
#pragma unroll
        for (int i = 0; i < kPkItems; ++i) {
            const uint64_t e = base + (uint64_t)i * kBlock + threadIdx.x;
            r1[i] = (e < m && x[i] + h < n) ? rank[x[i] + h] : 0u;
        }
#pragma unroll
        for (int i = 0; i < kPkItems; ++i) {
            const uint64_t e = base + (uint64_t)i * kBlock + threadIdx.x;
            if (e < m) {
                keys[e] = ((uint64_t)g[i] << wr) | r1[i];
                if (gp[i] != g[i]) {   // e == 0 or a group start
                    gs[g[i]] = (uint32_t)e;
                    pr[g[i]] = r1[i];
                }
                if (e == m - 1) gs[G] = (uint32_t)m;
            }
        }
    }
}

// where k_pivot_pass<3> puts the tied members (see the header)
struct TiedOut {
    const uint32_t* __restrict__ pos_in = nullptr;   // the round's u_pos: SA position per U slot
    const uint32_t* __restrict__ toff = nullptr;     // per group: next-set offset of its tied block
    const uint32_t* __restrict__ tid = nullptr;      // per group: the tied block's next-set group id
    uint32_t* __restrict__ rank = nullptr;
    uint32_t* __restrict__ sa = nullptr;
    uint32_t* __restrict__ u_pos = nullptr;
    uint32_t* __restrict__ u_idx = nullptr;
    uint32_t* __restrict__ u_g = nullptr;
    uint32_t* __restrict__ gsn = nullptr;            // the next set's group starts (or null)
};

// MODE 1's key source: key(e) = u_g[e] << wr | rank[u_idx[e] + h] (0 past
// the end), written to keys_out for the later passes; the pivot rank of
// each group to pr_out at its start
struct PivotKeySrc {
    const uint32_t* __restrict__ rank = nullptr;
    uint64_t n = 0, h = 0;
    uint64_t* __restrict__ keys_out = nullptr;
    uint32_t* __restrict__ pr_out = nullptr;
};

// MODE 0: cc[c * chunks + chunk] = members of class c in the chunk, and for
//         every group starting in the chunk gP[c * (G + 1) + g] = members of
//         class c before gs_g inside the chunk (k_pivot_gp adds the chunk's
//         scanned offset).
// MODE 2: tied members -> okeys / oidx at their final slots; the rest ->
//         rkeys / ridx at (members of classes 0 and 2 before them).
// MODE 3: the rest as MODE 2; tied members -> rank / sa / next set (TiedOut).
// MODE 1: MODE 0 with the keys built here (PivotKeySrc) instead of read:
//         k_pivot_keys and MODE 0 in one pass, when the group starts gs came
//         with the previous round's set (k_seg_write / MODE 3 wrote them)
// R1: round 1 (build_packed's pivot round 1): every suffix in one group, index
//     e itself, keys the packed K-symbol keys, pivot keys[0]; the rest keeps
//     its plain key (one group: key order already puts < p before > p).
template <int MODE, bool R1 = false>
__global__ __launch_bounds__(kBlock) void k_pivot_pass(const uint64_t* __restrict__ keys,
                                                       const uint32_t* __restrict__ u_idx,
                                                       const uint32_t* __restrict__ u_g, Chunking ch,
                                                       const uint32_t* __restrict__ gs, const uint32_t* __restrict__ pr,
                                                       uint32_t G, uint32_t wr,
                                                       uint32_t* __restrict__ cc, uint32_t* __restrict__ gP,
                                                       uint64_t* __restrict__ okeys, uint32_t* __restrict__ oidx,
                                                       uint64_t* __restrict__ rkeys, uint32_t* __restrict__ ridx,
                                                       TiedOut to = TiedOut{}, PivotKeySrc ks = PivotKeySrc{}) {
    constexpr bool COUNT = MODE == 0 || MODE == 1;
    __shared__ uint32_t s_w[3][kWaves];
    const uint32_t c = blockIdx.x;
    const uint64_t e0 = ch.begin(c), e1 = ch.end(c);
    const uint32_t wave = wave_id(), lane = lane_id();
    const uint64_t lt = lanemask_lt();
    uint32_t run[3] = {0, 0, 0};
    if (!COUNT)
        for (int k = 0; k < 3; ++k) run[k] = cc[(uint64_t)k * ch.chunks + c];
    const uint64_t gstride = (uint64_t)G + 1;
    const uint64_t p1 = R1 ? keys[0] : 0ull;
    // the per-group words of the lane's current group, reloaded only when its
    // group changes (U is in group order: a lane's groups only increase).  A
    // wave whose 1024 members lie in one group (first == last) loads them once,
    // outside the row loops, so its rows hold no load that a store must wait
    // for; other waves refresh them per member.
    uint32_t cg = ~0u, c_pr = 0, c_s0 = 0, c_cnt0 = 0, c_b1 = 0, c_cnt1 = 0, c_bp = 0, c_toff = 0, c_tid = 0;
    auto group = [&](uint32_t gg) {
        if (gg == cg) return;
        cg = gg;
        c_s0 = R1 ? 0u : gs[gg];
        if constexpr (MODE == 1) {   // the pivot: the key of the group's first member
            const uint64_t x0 = u_idx[c_s0];
            c_pr = x0 + ks.h < ks.n ? ks.rank[x0 + ks.h] : 0u;
        } else {
            c_pr = R1 ? 0u : pr[gg];
        }
        if (!COUNT) {
            c_cnt0 = gP[gg + 1] - gP[gg];
            c_b1 = gP[gstride + gg];
            c_cnt1 = gP[gstride + gg + 1] - c_b1;
        }
        if (MODE == 3) {
            c_bp = (R1 ? 0u : to.pos_in[c_s0]) + c_cnt0;   // the tied block's first SA position
            c_toff = to.toff[gg];
            c_tid = to.tid[gg];
        }
    };
    if (R1) group(0u);
    for (uint64_t tb = e0; tb < e1; tb += kTile) {
        const uint64_t w0 = tb + (uint64_t)wave * kWaveTile;
        uint64_t key[kItems];
        uint32_t g[kItems], xs[kItems];
        // every row's key and index loaded before any store (vmcnt counts
        // loads and stores in order: a load issued between stores would make
        // its row wait for them)
        if constexpr (MODE == 1) {
            // every row's index and group, then the rank gathers, then the keys
#pragma unroll
            for (int j = 0; j < kItems; ++j) {
                const uint64_t e = w0 + (uint64_t)j * kWave + lane;
                xs[j] = e < e1 ? u_idx[e] : 0u;
                g[j] = e < e1 ? u_g[e] : 0u;
            }
#pragma unroll
            for (int j = 0; j < kItems; ++j) {
                const uint64_t e = w0 + (uint64_t)j * kWave + lane;
                const uint64_t y = (uint64_t)xs[j] + ks.h;
                key[j] = ((uint64_t)g[j] << wr) | (e < e1 && y < ks.n ? ks.rank[y] : 0u);
            }
#pragma unroll
            for (int j = 0; j < kItems; ++j) {
                const uint64_t e = w0 + (uint64_t)j * kWave + lane;
                if (e < e1) ks.keys_out[e] = key[j];
            }
        } else {
#pragma unroll
            for (int j = 0; j < kItems; ++j) {
                const uint64_t e = w0 + (uint64_t)j * kWave + lane;
                key[j] = e < e1 ? keys[e] : 0ull;
                xs[j] = (MODE != 0 && !R1 && e < e1) ? u_idx[e] : (uint32_t)e;
                g[j] = (e < e1 && !R1) ? (uint32_t)(key[j] >> wr) : 0u;   // key = g << wr | rank
            }
        }
        bool uni = true;
        if (!R1) {
            const uint32_t g0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)g[0]);
            uint64_t diff = 0;
#pragma unroll
            for (int j = 0; j < kItems; ++j) diff |= __ballot(w0 + (uint64_t)j * kWave + lane < e1 && g[j] != g0);
            uni = diff == 0;
            if (uni) group(g0);
        }
        uint32_t cls[kItems];
        uint32_t wc[3] = {0, 0, 0};
        auto classify = [&](auto uni_tag) {
#pragma unroll
            for (int j = 0; j < kItems; ++j) {
                const uint64_t e = w0 + (uint64_t)j * kWave + lane;
                if (!decltype(uni_tag)::value && e < e1) group(g[j]);
                const uint64_t p = R1 ? p1 : e < e1 ? (((uint64_t)g[j] << wr) | c_pr) : 0ull;
                cls[j] = e < e1 ? (key[j] < p ? 0u : key[j] == p ? 1u : 2u) : 3u;
#pragma unroll
                for (int k = 0; k < 3; ++k) wc[k] += (uint32_t)__popcll(__ballot(cls[j] == (uint32_t)k));
            }
        };
        if (uni)
            classify(std::true_type{});
        else
            classify(std::false_type{});
        if (lane == 0)
            for (int k = 0; k < 3; ++k) s_w[k][wave] = wc[k];
        __syncthreads();
        uint32_t off[3], tot[3];
        for (int k = 0; k < 3; ++k) {
            off[k] = run[k];
            tot[k] = 0;
            for (int w = 0; w < kWaves; ++w) {
                const uint32_t v = s_w[k][w];
                off[k] += (w < (int)wave) ? v : 0u;
                tot[k] += v;
            }
        }
        auto scatter = [&](auto uni_tag) {
#pragma unroll
            for (int j = 0; j < kItems; ++j) {
                const uint64_t e = w0 + (uint64_t)j * kWave + lane;
                uint64_t bm[3];
#pragma unroll
                for (int k = 0; k < 3; ++k) bm[k] = __ballot(cls[j] == (uint32_t)k);
                if (e < e1) {
                    // P_c(e): members of class c before e
                    const uint32_t P0 = off[0] + (uint32_t)__popcll(bm[0] & lt);
                    const uint32_t P1 = off[1] + (uint32_t)__popcll(bm[1] & lt);
                    const uint32_t P2 = off[2] + (uint32_t)__popcll(bm[2] & lt);
                    const uint32_t gg = g[j];
                    if (!decltype(uni_tag)::value) group(gg);
                    if (COUNT) {
                        if (c_s0 == (uint32_t)e) {   // in-chunk counts before the group start
                            gP[gg] = P0;
                            gP[gstride + gg] = P1;
                            gP[2 * gstride + gg] = P2;
                            if (MODE == 1) ks.pr_out[gg] = (uint32_t)(key[j] & ((1ull << wr) - 1ull));
                        }
                    } else {
                        const uint32_t x = xs[j];
                        if (MODE == 3 && cls[j] == 1u) {
                            const uint32_t t = P1 - c_b1;
                            to.rank[x] = c_bp + 1u;
                            if (c_cnt1 == 1u) {
                                to.sa[c_bp] = x;
                            } else {
                                const uint32_t q = c_toff + t;
                                to.u_pos[q] = c_bp + t;
                                to.u_idx[q] = x;
                                to.u_g[q] = c_tid;
                                if (to.gsn && t == 0u) to.gsn[c_tid] = q;
                            }
                        } else if (cls[j] == 1u) {
                            const uint64_t ne = (uint64_t)c_s0 + c_cnt0 + (P1 - c_b1);
                            okeys[ne] = key[j];
                            oidx[ne] = x;
                        } else {
                            const uint64_t ri = (uint64_t)P0 + P2;
                            rkeys[ri] = R1 ? key[j]
                                           : ((uint64_t)(2u * gg + (cls[j] == 2u ? 1u : 0u)) << wr) |
                                                 (key[j] & ((1ull << wr) - 1ull));
                            ridx[ri] = x;
                        }
                    }
                }
#pragma unroll
                for (int k = 0; k < 3; ++k) off[k] += (uint32_t)__popcll(bm[k]);
            }
        };
        if (uni)
            scatter(std::true_type{});
        else
            scatter(std::false_type{});
        for (int k = 0; k < 3; ++k) run[k] += tot[k];
        __syncthreads();
    }
    if (COUNT && threadIdx.x == 0)
        for (int k = 0; k < 3; ++k) cc[(uint64_t)k * ch.chunks + c] = run[k];
}

// gP[c][g] += the scanned class-c count before the chunk holding gs_g;
// gP[c][G] = the class totals (one thread per group)
__global__ __launch_bounds__(kBlock) void k_pivot_gp(const uint32_t* __restrict__ gs, uint32_t G,
                                                     const uint32_t* __restrict__ cc, Chunking ch,
                                                     const uint32_t* __restrict__ totals, uint32_t* __restrict__ gP) {
    const uint64_t gstride = (uint64_t)G + 1;
    const uint64_t csize = (uint64_t)ch.tiles_per_chunk * kTile;
    for (uint64_t g = (uint64_t)blockIdx.x * kBlock + threadIdx.x; g <= G; g += (uint64_t)gridDim.x * kBlock) {
        if (g == G) {
            for (int k = 0; k < 3; ++k) gP[k * gstride + G] = totals[k];
        } else {
            const uint64_t chunk = gs[g] / csize;
            for (int k = 0; k < 3; ++k) gP[k * gstride + g] += cc[(uint64_t)k * ch.chunks + chunk];
        }
    }
}

// toff[g] / tid[g] (k_pivot_pass<3>): exclusive scans over the groups of the
// tied block sizes of two or more and of the number of such blocks;
// totals[0..2] = (members of such blocks, such blocks, nonempty blocks).  One
// workgroup (pivot_round takes this path for G <= kPivotTiedMaxG only).
__global__ __launch_bounds__(kBlock) void k_pivot_tied_scan(const uint32_t* __restrict__ gP, uint32_t G,
                                                            uint32_t* __restrict__ toff, uint32_t* __restrict__ tid,
                                                            uint32_t* __restrict__ totals) {
    __shared__ uint32_t s_tmp[kWaves];
    const uint32_t* const g1 = gP + (uint64_t)G + 1;   // class-1 members before each group
    uint32_t ct = 0, cb = 0, cd = 0;
    for (uint32_t base = 0; base < G; base += kBlock * 4) {
        uint32_t vt[4], vb[4], st = 0, sb = 0, sd = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t i = base + threadIdx.x * 4 + j;
            const uint32_t cnt = i < G ? g1[i + 1] - g1[i] : 0u;
            vt[j] = cnt >= 2u ? cnt : 0u;
            vb[j] = cnt >= 2u ? 1u : 0u;
            st += vt[j];
            sb += vb[j];
            sd += cnt ? 1u : 0u;
        }
        uint32_t tt, tb, td;
        uint32_t ot = block_exclusive_sum(st, s_tmp, &tt) + ct;
        uint32_t ob = block_exclusive_sum(sb, s_tmp, &tb) + cb;
        (void)block_exclusive_sum(sd, s_tmp, &td);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t i = base + threadIdx.x * 4 + j;
            if (i < G) {
                toff[i] = ot;
                tid[i] = ob;
            }
            ot += vt[j];
            ob += vb[j];
        }
        ct += tt;
        cb += tb;
        cd += td;
    }
    if (threadIdx.x == 0) {
        totals[0] = ct;
        totals[1] = cb;
        totals[2] = cd;
    }
}

// the sorted rest (keys (2 g + [> p]) << wr | rank) to the final slots of
// their group: class 0 first, class 2 after the tied block.  POS: only each
// member's SA position, rpos[j] = pos_in[slot] (the tied-block round keeps
// the rest in sorted order and runs segments() over it).
template <bool POS>
__global__ __launch_bounds__(kBlock) void k_pivot_place(const uint64_t* __restrict__ rkeys,
                                                        const uint32_t* __restrict__ ridx, uint64_t mr,
                                                        const uint32_t* __restrict__ gs,
                                                        const uint32_t* __restrict__ gP, uint32_t G, uint32_t wr,
                                                        uint64_t* __restrict__ okeys, uint32_t* __restrict__ oidx,
                                                        uint64_t m, const uint32_t* __restrict__ pos_in = nullptr,
                                                        uint32_t* __restrict__ rpos = nullptr) {
    const uint64_t gstride = (uint64_t)G + 1;
    for (uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x; j < mr; j += (uint64_t)gridDim.x * kBlock) {
        const uint64_t k = rkeys[j];
        const uint32_t sub = (uint32_t)(k >> wr);
        const uint32_t g = sub >> 1;
        if (g >= G) continue;
        const uint32_t R = gP[g] + gP[2 * gstride + g];           // rest members before group g
        const uint32_t cnt1 = gP[gstride + g + 1] - gP[gstride + g];
        const uint64_t ne = (sub & 1u) ? (uint64_t)gs[g] + cnt1 + (j - R) : (uint64_t)gs[g] + (j - R);
        if (ne < m) {
            if (POS) {
                rpos[j] = pos_in[ne];
            } else {
                okeys[ne] = ((uint64_t)g << wr) | (k & ((1ull << wr) - 1ull));
                oidx[ne] = ridx[j];
            }
        }
    }
}

}  // namespace sa
