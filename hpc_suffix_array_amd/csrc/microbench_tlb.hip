// microbench_tlb.hip -- is the bucket passes' speed set by how far apart
// their write destinations lie?  A pass shaped like the second bucket pass
// (12288 items per tile read in order, written as 512 runs of 24) with the
// 512 destination regions either spread over the whole output (the second
// pass: bucket (h, l) for all h of one segment l) or packed into one
// 64 MiB window per group of 341 tiles (an l-major layout), each timed on
// several fresh allocations of the output buffer.  Not part of libsa_hip.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

constexpr int B = 1024, IT = 12, T = B * IT, R = 512, RUN = T / R;   // 24
constexpr int TPG = 341;                                               // tiles per group (one segment)

__global__ __launch_bounds__(B) void k_pass(const uint64_t* __restrict__ in, uint64_t* __restrict__ out,
                                            uint64_t n, int local) {
    const uint64_t tiles = n / T;
    const uint64_t per_region = n / R;   // spread layout: region r = [r per_region, ...)
    for (uint64_t t = blockIdx.x; t < tiles; t += gridDim.x) {
        uint64_t v[IT];
#pragma unroll
        for (int j = 0; j < IT; ++j) v[j] = in[t * T + j * B + threadIdx.x];
#pragma unroll
        for (int j = 0; j < IT; ++j) {
            const uint32_t q = j * B + threadIdx.x;      // item q of the tile -> run q / RUN
            const uint32_t r = q / RUN, k = q % RUN;
            uint64_t dst;
            if (local) {   // group g's 512 regions side by side: RUN * TPG items each
                const uint64_t g = t / TPG, tg = t % TPG;
                dst = (g * R + r) * (uint64_t)(RUN * TPG) + tg * RUN + k;
            } else {
                dst = r * per_region + t * RUN + k;
            }
            if (dst < n) out[dst] = v[j] + 1;
        }
    }
}

int main(int argc, char** argv) {
    const bool skip_offsets = argc > 1;   // any argument: allocations only
    const uint64_t n = 1ull << 30;
    uint64_t* in;
    CK(hipMalloc(&in, n * 8));
    CK(hipMemset(in, 1, n * 8));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    // one allocation, the output at different offsets inside it: address
    // bits below the page (channel / bank interleave) vs the pages themselves
    if (!skip_offsets) {
        uint64_t* big;
        CK(hipMalloc(&big, n * 8 + (64ull << 20)));
        for (uint64_t off : {0ull, 4096ull, 65536ull, 1ull << 21, 3ull << 21, 1ull << 25}) {
            uint64_t* out = big + off / 8;
            std::vector<float> ts;
            for (int r = 0; r < 4; ++r) {
                CK(hipEventRecord(a));
                hipLaunchKernelGGL(k_pass, dim3(cus), dim3(B), 0, 0, (const uint64_t*)in, out, n, 0);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                ts.push_back(ms);
            }
            std::sort(ts.begin(), ts.end());
            std::printf("one allocation, output at +%llu B, spread: %.3f ms\n", (unsigned long long)off, ts[1]);
        }
        CK(hipFree(big));
    }
    std::vector<uint64_t*> keep;
    // allocations alternate between hipMalloc and hipExtMallocWithFlags(
    // hipDeviceMallocContiguous) (physically contiguous pages)
    for (int alloc = 0; alloc < 10; ++alloc) {
        uint64_t* out;
        const bool contig = alloc & 1;
        if (contig) CK(hipExtMallocWithFlags((void**)&out, n * 8, hipDeviceMallocContiguous));
        else CK(hipMalloc(&out, n * 8));
        keep.push_back(out);   // a new allocation every time (the old ones stay mapped)
        for (int local = 0; local < 2; ++local) {
            std::vector<float> ts;
            for (int r = 0; r < 4; ++r) {
                CK(hipEventRecord(a));
                hipLaunchKernelGGL(k_pass, dim3(cus), dim3(B), 0, 0, (const uint64_t*)in, out, n, local);
                CK(hipEventRecord(b));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                ts.push_back(ms);
            }
            std::sort(ts.begin(), ts.end());
            std::printf("allocation %d %s %s: %.3f ms (%.0f GB/s)\n", alloc, contig ? "contiguous" : "hipMalloc ",
                        local ? "local 64 MiB windows" : "spread over 8 GiB  ",
                        ts[1], 16.0 * n / ts[1] / 1e6);
        }
        if (keep.size() >= 3) {   // bounded memory: free the oldest
            CK(hipFree(keep.front()));
            keep.erase(keep.begin());
        }
    }
    return 0;
}
