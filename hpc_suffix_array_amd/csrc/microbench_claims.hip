// microbench_claims.hip -- throughput of the bucket passes' per-tile claims:
// every tile adds its per-digit counts to RADIX device-scope cursors with
// one atomic per digit (k_split_text: 256 cursors shared by every tile;
// k_split_seg: one cursor per (segment, digit)).  Measures the claims alone
// (no data), for T tiles over W persistent workgroups, with the cursors
// shared (S = 1) or striped over S copies (tile t uses copy t % S).
// Not part of libsa_hip.
//   build: hipcc -O3 --offload-arch=gfx950 microbench_claims.hip -o microbench_claims
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

__global__ __launch_bounds__(512) void k_claims(uint32_t* cur, uint32_t* ticket, uint32_t tiles, uint32_t radix,
                                                uint32_t stripes, uint32_t* sink) {
    __shared__ uint32_t s_t;
    uint32_t acc = 0;
    for (;;) {
        if (threadIdx.x == 0) s_t = atomicAdd(ticket, 1u);
        __syncthreads();
        const uint32_t t = s_t;
        __syncthreads();
        if (t >= tiles) break;
        // stripes > 0: row t % stripes; stripes == 0: row t / per_seg (the
        // second pass: consecutive units share a segment's cursors)
        const uint32_t row = stripes ? t % stripes : (t / 341u) % 256u;
        if (threadIdx.x < radix) acc += atomicAdd(&cur[row * radix + threadIdx.x], 24u);
        __syncthreads();
    }
    if (acc == 0xFFFFFFFFu) sink[0] = acc;
}

int main(int argc, char** argv) {
    const uint32_t tiles = argc > 1 ? std::atoi(argv[1]) : 174763;
    uint32_t *cur, *tick, *sink;
    CK(hipMalloc(&cur, 256 * 1024 * 4));
    CK(hipMalloc(&tick, 4));
    CK(hipMalloc(&sink, 4));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (uint32_t radix : {256u, 512u}) {
        for (uint32_t stripes : {1u, 8u, 64u, 0u}) {
            for (int wpc : {1, 2}) {
                std::vector<float> t;
                for (int r = 0; r < 4; ++r) {
                    CK(hipMemset(cur, 0, 256 * 1024 * 4));
                    CK(hipMemset(tick, 0, 4));
                    CK(hipEventRecord(a));
                    hipLaunchKernelGGL(k_claims, dim3(cus * wpc), dim3(512), 0, 0, cur, tick, tiles, radix, stripes, sink);
                    CK(hipEventRecord(b));
                    CK(hipEventSynchronize(b));
                    float ms;
                    CK(hipEventElapsedTime(&ms, a, b));
                    t.push_back(ms);
                }
                std::sort(t.begin(), t.end());
                std::printf("tiles %u radix %u stripes %2u wg/cu %d: %.3f ms (%.1f ns per tile)\n", tiles, radix,
                            stripes, wpc, t[1], t[1] * 1e6 / tiles);
            }
        }
    }
    return 0;
}
