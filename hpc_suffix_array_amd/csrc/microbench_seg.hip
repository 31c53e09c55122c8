// microbench_seg.hip -- the second bucket pass's write pattern, isolated:
// 2^30 packed 8-byte items in 256 input segments (the first pass's digit l),
// each item's 9-bit digit h on top (uniform random); persistent workgroups
// take units (TILE items of one segment) from a ticket, rank the items by
// LDS atomics, claim each digit's run from an atomic cursor, stage the unit
// digit-sorted in LDS and write the runs -- k_split_seg without its base
// chain (the bases are exact, precomputed outside the timed region).
//   layout 0 (k_split_seg): one output in bucket order (h, l); one ticket;
//            cursor (l, h); a run's neighbours come from whichever units
//            claimed just before / after it, on any XCD.
//   layout 1 (per-XCD regions): unit u belongs to queue x = u mod 8, served
//            by the workgroups w with w mod 8 = x (one XCD each: workgroups
//            are dealt to the 8 XCDs round robin); the output holds 8
//            regions, region x in bucket order over queue x's items, cursor
//            (x, l, h): a run's neighbours are written by the same XCD, whose
//            L2 can merge the partial lines at the runs' ends.
// ITEMS 12 (tile 12288: runs of ~24 items) and 16 (tile 16384: ~32).
// Not part of libsa_hip.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

constexpr int B = 1024, R = 512, S = 256, X = 8;
constexpr uint32_t SH = 55;   // digit h = item >> SH

__device__ __forceinline__ void unit_of(uint64_t u, uint64_t upl, uint64_t seg, uint32_t T, uint32_t& l, uint64_t& tb,
                                        uint32_t& valid) {
    l = (uint32_t)(u / upl);
    const uint64_t i = u % upl;
    tb = (uint64_t)l * seg + i * T;
    const uint64_t e = (uint64_t)(l + 1) * seg;
    valid = (uint32_t)std::min<uint64_t>(T, e - tb);
}

// counts per (queue, l, h) of the unit assignment (not timed)
template <int IT>
__global__ void k_count(const uint64_t* __restrict__ in, uint64_t n, uint64_t upl, uint64_t seg, int layout,
                        uint32_t* __restrict__ cnt) {
    constexpr uint32_t T = B * IT;
    const uint64_t units = upl * S;
    for (uint64_t u = blockIdx.x; u < units; u += gridDim.x) {
        uint32_t l, valid;
        uint64_t tb;
        unit_of(u, upl, seg, T, l, tb, valid);
        const uint32_t x = layout ? (uint32_t)(u % X) : 0u;
        for (uint32_t q = threadIdx.x; q < valid; q += B)
            atomicAdd(&cnt[((uint64_t)x * S + l) * R + (in[tb + q] >> SH)], 1u);
    }
}

template <int IT>
__global__ __launch_bounds__(B) void k_seg(const uint64_t* __restrict__ in, uint64_t n, uint64_t upl, uint64_t seg,
                                           int layout, const uint32_t* __restrict__ base, uint32_t* __restrict__ cur,
                                           uint32_t* __restrict__ tickets, uint64_t* __restrict__ out) {
    constexpr uint32_t T = B * IT;
    __shared__ uint64_t s_keys[T];
    __shared__ uint32_t s_cnt[R];
    __shared__ uint32_t s_start[R];
    __shared__ uint32_t s_gofs[R];
    __shared__ uint32_t s_tmp[B / 64];
    __shared__ uint32_t s_t;
    const uint32_t dg = threadIdx.x, lane = dg & 63, wave = dg >> 6;
    const uint32_t x = layout ? blockIdx.x % X : 0u;
    const uint64_t units = upl * S;
    const uint64_t qunits = layout ? (units - x + X - 1) / X : units;   // units of queue x
    uint32_t* const ticket = tickets + x * 32;
    for (;;) {
        if (dg < R) s_cnt[dg] = 0;
        if (dg == 0) s_t = atomicAdd(ticket, 1u);
        __syncthreads();
        const uint64_t t = s_t;
        if (t >= qunits) break;
        const uint64_t u = layout ? t * X + x : t;
        uint32_t l, valid;
        uint64_t tb;
        unit_of(u, upl, seg, T, l, tb, valid);
        uint64_t k[IT];
        uint32_t dr[IT];
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            const uint32_t le = wave * 64 * IT + j * 64 + lane;
            k[j] = in[tb + (le < valid ? le : valid - 1)];
        }
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            const uint32_t le = wave * 64 * IT + j * 64 + lane;
            const uint32_t d = le < valid ? (uint32_t)(k[j] >> SH) : (uint32_t)R;
            dr[j] = (d << 16) | (d < R ? atomicAdd(&s_cnt[d], 1u) : 0u);
        }
        __syncthreads();
        uint32_t c = 0;
        if (dg < R) {
            c = s_cnt[dg];
            const uint64_t ci = ((uint64_t)x * S + l) * R + dg;
            s_gofs[dg] = base[ci] + (c ? atomicAdd(&cur[ci], c) : 0u);
        }
        {   // exclusive scan of the counts (8 waves of 64 digits)
            uint32_t inc = c;
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(inc, o, 64);
                if ((int)lane >= o) inc += y;
            }
            if (lane == 63 && wave < R / 64) s_tmp[wave] = inc;
            __syncthreads();
            uint32_t off = 0;
            for (uint32_t w = 0; w < wave && w < R / 64; ++w) off += s_tmp[w];
            if (dg < R) s_start[dg] = off + inc - c;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            const uint32_t d = dr[j] >> 16;
            if (d < R) s_keys[s_start[d] + (dr[j] & 0xFFFFu)] = k[j];
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            const uint32_t q = j * B + dg;
            if (q < valid) {
                const uint64_t w = s_keys[q];
                const uint32_t d = (uint32_t)(w >> SH);
                out[(uint64_t)s_gofs[d] + (q - s_start[d])] = w & ((1ull << SH) - 1);
            }
        }
        __syncthreads();
    }
}

static uint64_t rng_state = 12345;
static uint64_t splitmix() {
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

template <int IT>
static void run(const uint64_t* d_in, uint64_t* d_out, uint64_t n, int grid, int layout) {
    constexpr uint32_t T = B * IT;
    const uint64_t seg = n / S, upl = (seg + T - 1) / T;
    const uint64_t ncnt = (uint64_t)X * S * R;
    uint32_t *d_cnt, *d_base, *d_cur, *d_tk;
    CK(hipMalloc(&d_cnt, ncnt * 4));
    CK(hipMalloc(&d_base, ncnt * 4));
    CK(hipMalloc(&d_cur, ncnt * 4));
    CK(hipMalloc(&d_tk, X * 32 * 4));
    CK(hipMemset(d_cnt, 0, ncnt * 4));
    hipLaunchKernelGGL((k_count<IT>), dim3(4096), dim3(B), 0, 0, d_in, n, upl, seg, layout, d_cnt);
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> cnt(ncnt), base(ncnt);
    CK(hipMemcpy(cnt.data(), d_cnt, ncnt * 4, hipMemcpyDeviceToHost));
    // region x in bucket order (h, l); regions side by side
    uint64_t pos = 0;
    for (int x = 0; x < X; ++x)
        for (int h = 0; h < R; ++h)
            for (int l = 0; l < S; ++l) {
                const uint64_t i = ((uint64_t)x * S + l) * R + h;
                base[i] = (uint32_t)pos;
                pos += cnt[i];
            }
    if (pos != n) { std::printf("count mismatch %llu\n", (unsigned long long)pos); std::exit(1); }
    CK(hipMemcpy(d_base, base.data(), ncnt * 4, hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<float> ts;
    for (int rep = 0; rep < 7; ++rep) {
        CK(hipMemset(d_cur, 0, ncnt * 4));
        CK(hipMemset(d_tk, 0, X * 32 * 4));
        CK(hipEventRecord(a));
        hipLaunchKernelGGL((k_seg<IT>), dim3(grid), dim3(B), 0, 0, d_in, n, upl, seg, layout, d_base, d_cur, d_tk,
                           d_out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        ts.push_back(ms);
    }
    // check: every written item is a source item (sum of the low bits)
    std::sort(ts.begin(), ts.end());
    std::printf("layout %d (%s) tile %5u (runs ~%4.1f items): median %.3f ms  min %.3f  %.0f GB/s\n", layout,
                layout ? "per-XCD regions" : "one region     ", T, (double)T / R, ts[3], ts[0], 16.0 * n / ts[3] / 1e6);
    CK(hipFree(d_cnt));
    CK(hipFree(d_base));
    CK(hipFree(d_cur));
    CK(hipFree(d_tk));
}

int main() {
    const uint64_t n = 1ull << 30;
    std::vector<uint64_t> h(n);
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t r = splitmix();
        h[i] = ((r >> 7) & ((1ull << SH) - 1)) | ((r & 511ull) << SH);
    }
    uint64_t *in, *out;
    CK(hipMalloc(&in, n * 8));
    CK(hipMalloc(&out, n * 8));
    CK(hipMemcpy(in, h.data(), n * 8, hipMemcpyHostToDevice));
    CK(hipMemset(out, 0, n * 8));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    std::printf("CUs %d\n", cus);
    for (int pass = 0; pass < 2; ++pass) {
        run<12>(in, out, n, cus, 0);
        run<12>(in, out, n, cus, 1);
        run<16>(in, out, n, cus, 0);
        run<16>(in, out, n, cus, 1);
    }
    return 0;
}
