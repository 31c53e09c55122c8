// microbench_runs.hip -- how fast does a pass write 2^30 8-byte items when
// each tile of T items leaves as R runs of T / R items (the bucket passes:
// T = 12288, R = 512 in the second pass, 6144 / 256 in the first)?  The
// same kernel shape as microbench_tlb.hip's "spread" layout (region r of R
// spans n / R items of the output), swept over the run length, on one
// output allocation; R = 1 is a streaming copy.  xmaj: tiles dealt to
// XCDs in contiguous blocks (block b takes tiles of XCD b % 8 in order), so
// that a region's consecutive chunks are written by one XCD (one L2); else
// tile t on block t % grid (consecutive tiles on different XCDs).  Not part
// of libsa_hip.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

template <int B, int IT>
__global__ __launch_bounds__(B) void k_pass(const uint64_t* __restrict__ in, uint64_t* __restrict__ out, uint64_t n,
                                            uint32_t R, int xmaj) {
    constexpr uint32_t T = B * IT;
    const uint32_t run = T / R;
    const uint64_t tiles = n / T;
    const uint64_t per_region = n / R;
    const uint64_t per_xcd = tiles / 8, blocks_xcd = gridDim.x / 8;
    for (uint64_t k = 0;; ++k) {
        uint64_t t;
        if (xmaj) {
            const uint64_t i = blockIdx.x / 8 + k * blocks_xcd;
            if (i >= per_xcd) break;
            t = (blockIdx.x % 8) * per_xcd + i;
        } else {
            t = blockIdx.x + k * gridDim.x;
            if (t >= tiles) break;
        }
        uint64_t v[IT];
#pragma unroll
        for (int j = 0; j < IT; ++j) v[j] = in[t * T + j * B + threadIdx.x];
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            const uint32_t q = j * B + threadIdx.x;
            const uint32_t r = q / run, k = q % run;
            const uint64_t dst = r * per_region + t * run + k;
            if (dst < n) out[dst] = v[j] + 1;
        }
    }
}

template <int B, int IT>
static void sweep(const uint64_t* in, uint64_t* out, uint64_t n, int grid, hipEvent_t a, hipEvent_t b) {
    constexpr uint32_t T = B * IT;
    for (int xmaj = 0; xmaj < 2; ++xmaj)
    for (uint32_t R : {1u, 64u, 128u, 256u, 512u, 1024u, 2048u}) {
        if (T % R) continue;
        std::vector<float> ts;
        for (int rep = 0; rep < 5; ++rep) {
            CK(hipEventRecord(a));
            hipLaunchKernelGGL((k_pass<B, IT>), dim3(grid), dim3(B), 0, 0, in, out, n, R, xmaj);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            ts.push_back(ms);
        }
        std::sort(ts.begin(), ts.end());
        std::printf("%s block %4d x %2d (tile %5u) regions %4u run %5u items (%6u B): %.3f ms  %.0f GB/s\n",
                    xmaj ? "xcd-major  " : "round-robin", B, IT, T, R, T / R, 8 * T / R, ts[2], 16.0 * n / ts[2] / 1e6);
    }
}

int main() {
    const uint64_t n = 1ull << 30;
    uint64_t *in, *out;
    CK(hipMalloc(&in, n * 8));
    CK(hipMalloc(&out, n * 8));
    CK(hipMemset(in, 1, n * 8));
    CK(hipMemset(out, 0, n * 8));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    sweep<1024, 12>(in, out, n, cus, a, b);       // the second pass's shape
    sweep<1024, 16>(in, out, n, cus, a, b);
    sweep<512, 12>(in, out, n, 2 * cus, a, b);    // the first pass's shape (two per CU)
    sweep<1024, 8>(in, out, n, 2 * cus, a, b);
    return 0;
}
