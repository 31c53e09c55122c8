// sa_build.hip -- host driver of the MI355X rank-doubling suffix-array
// builder and the extended C ABI of include/sa_hip.h.
//
// Round structure (replaces build_suffix_array, manber_myers.c:81-133):
//   rank_1 = text + 1                                   (k_init_rank)
//   for h = 1, 2, 4, ...:                               (:97, 64-bit bound)
//     w  = bit width of D (ranks are 0..D)
//     P  = ceil(2w / 8) LSD passes over key (rank[i] << w) | rank[i+h]
//          pass 0 builds the key from ranks (the :116-124 update, fused)
//     D' = number of distinct keys                      (k_heads, k_scan_heads)
//     stop when D' == n                                 (:113)
//     rank[idx[p]] = dense rank of p                    (k_rerank, :101-110)
// The caller's SA buffer is one of the two index ping-pong buffers, chosen
// per round by the parity of P so the last pass writes the SA in place.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/sa_hip.h"
#include "sa_kernels.h"

namespace sa {

static thread_local std::string g_err;

static int set_err(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define SA_HIP(call)                                                                         \
    do {                                                                                     \
        hipError_t e_ = (call);                                                              \
        if (e_ != hipSuccess)                                                                \
            return set_err(SA_E_HIP, "%s failed: %s (%s:%d)", #call, hipGetErrorString(e_),  \
                           __FILE__, __LINE__);                                              \
    } while (0)

static bool trace_on() {
    static const bool on = std::getenv("SA_TRACE") != nullptr;
    return on;
}
#define SA_TRACE(...)                                   \
    do {                                                \
        if (trace_on()) {                               \
            std::fprintf(stderr, "[sa] " __VA_ARGS__);  \
            std::fputc('\n', stderr);                   \
        }                                               \
    } while (0)

constexpr uint32_t kMaxChunks = 1024;
constexpr int kEvPool = 256;

static uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

static uint32_t bit_width(uint64_t x) {
    uint32_t w = 0;
    while (x) { ++w; x >>= 1; }
    return w;
}

static Chunking plan_chunks(uint64_t n) {
    Chunking ch;
    ch.n = n;
    const uint64_t tiles = (n + kTile - 1) / kTile;
    uint64_t tpc = (tiles + kMaxChunks - 1) / kMaxChunks;
    if (tpc == 0) tpc = 1;
    ch.tiles_per_chunk = (uint32_t)tpc;
    ch.chunks = (uint32_t)std::max<uint64_t>(1, (tiles + tpc - 1) / tpc);
    return ch;
}

}  // namespace sa

struct sa_context {
    int device = 0;
    uint64_t cap = 0;
    uint32_t* rank = nullptr;
    uint64_t* keys[2] = {nullptr, nullptr};
    uint32_t* vals_alt = nullptr;
    uint32_t* hist = nullptr;      // 256 * kMaxChunks
    uint32_t* totals = nullptr;    // 256
    uint32_t* counts = nullptr;    // kMaxChunks
    uint32_t* words = nullptr;     // [0] = D, [1] = check error flags
    uint32_t* host_words = nullptr;  // pinned mirror
    hipEvent_t ev[sa::kEvPool];
    int ev_ready = 0;
};

namespace sa {

// Device memory a context holds for n symbols (rank + 2 key + 1 index buffer).
static uint64_t ws_bytes(uint64_t n) {
    const uint64_t m = align_up(std::max<uint64_t>(n, 1), 64);
    return m * 4 + 2 * m * 8 + m * 4 + (uint64_t)kRadix * kMaxChunks * 4 + 4096;
}

static void free_ctx_buffers(sa_context* c) {
    hipFree(c->rank);
    hipFree(c->keys[0]);
    hipFree(c->keys[1]);
    hipFree(c->vals_alt);
    c->rank = nullptr;
    c->keys[0] = c->keys[1] = nullptr;
    c->vals_alt = nullptr;
    c->cap = 0;
}

static int ensure_capacity(sa_context* c, uint64_t n) {
    if (n <= c->cap && c->rank) return SA_OK;
    SA_HIP(hipSetDevice(c->device));
    free_ctx_buffers(c);
    const uint64_t m = align_up(std::max<uint64_t>(n, 1), 64);
    if (hipMalloc(&c->rank, m * 4) != hipSuccess || hipMalloc(&c->keys[0], m * 8) != hipSuccess ||
        hipMalloc(&c->keys[1], m * 8) != hipSuccess || hipMalloc(&c->vals_alt, m * 4) != hipSuccess) {
        free_ctx_buffers(c);
        (void)hipGetLastError();
        return set_err(SA_E_NOMEM, "device allocation of %.2f GiB workspace failed",
                       (double)ws_bytes(n) / (1ull << 30));
    }
    c->cap = n;
    return SA_OK;
}

// Per-launch HIP-event timing, enabled by sa_opts.profile.
struct Timer {
    sa_context* c;
    hipStream_t s;
    bool on;
    int used = 0;
    int kind[kEvPool / 2];
    sa_stats* st;
    void begin(int k) {
        if (!on) return;
        if (used >= kEvPool / 2) flush();
        kind[used] = k;
        hipEventRecord(c->ev[2 * used], s);
    }
    void end() {
        if (!on) return;
        hipEventRecord(c->ev[2 * used + 1], s);
        ++used;
    }
    void flush() {
        if (!on || used == 0) return;
        hipEventSynchronize(c->ev[2 * used - 1]);
        for (int i = 0; i < used; ++i) {
            float ms = 0.f;
            hipEventElapsedTime(&ms, c->ev[2 * i], c->ev[2 * i + 1]);
            if (st) {
                st->kern_ms[kind[i]] += ms;
                st->kern_launches[kind[i]] += 1;
            }
        }
        used = 0;
    }
};

static void add_bytes(sa_stats* st, int kind, uint64_t b) {
    if (st) st->kern_bytes[kind] += b;
}

// One LSD radix pass over bits [shift, shift + nbits).
template <class Src>
static int radix_pass(sa_context* c, const Src& src, const Chunking& ch, uint32_t shift, uint32_t nbits,
                      uint64_t* out_keys, uint32_t* out_vals, hipStream_t s, Timer& tm, sa_stats* st,
                      int kind_hist, int kind_scatter, uint64_t in_bytes) {
    const uint32_t mask = (1u << nbits) - 1u;
    tm.begin(kind_hist);
    hipLaunchKernelGGL(k_hist<Src>, dim3(ch.chunks), dim3(kBlock), 0, s, src, ch, shift, mask, c->hist);
    tm.end();
    tm.begin(SA_K_SCAN);
    hipLaunchKernelGGL(k_scan_rows, dim3(kRadix), dim3(kBlock), 0, s, c->hist, ch.chunks, c->totals);
    tm.end();
    tm.begin(kind_scatter);
    hipLaunchKernelGGL(k_scatter<Src>, dim3(ch.chunks), dim3(kBlock), 0, s, src, ch, shift, nbits,
                       (const uint32_t*)c->hist, (const uint32_t*)c->totals, out_keys, out_vals);
    tm.end();
    SA_HIP(hipGetLastError());
    add_bytes(st, kind_hist, in_bytes);
    add_bytes(st, SA_K_SCAN, 2ull * 4 * kRadix * ch.chunks);
    add_bytes(st, kind_scatter, in_bytes + 12ull * ch.n);
    return SA_OK;
}

static int build_device(sa_context* c, const uint8_t* d_text, uint64_t n, uint32_t* d_sa, hipStream_t s,
                        const sa_opts* opts, sa_stats* st) {
    if (st) {
        std::memset(st, 0, sizeof *st);
        st->n_kinds = SA_K_COUNT;
    }
    if (n == 0) return SA_OK;
    if (!d_text || !d_sa) return set_err(SA_E_INVALID, "NULL device pointer");
    if (n > 0xFFFFFFFFull) return set_err(SA_E_INVALID, "n = %llu exceeds 2^32-1 on one device",
                                          (unsigned long long)n);
    SA_HIP(hipSetDevice(c->device));
    int rc = ensure_capacity(c, n);
    if (rc) return rc;
    Timer tm{c, s, opts && opts->profile, 0, {}, st};

    // round / whole-build events (the pool's events are reserved for Timer)
    hipEvent_t r0, r1, start_all;
    SA_HIP(hipEventCreate(&r0));
    SA_HIP(hipEventCreate(&r1));
    SA_HIP(hipEventCreate(&start_all));
    SA_HIP(hipEventRecord(start_all, s));

    SA_TRACE("build n=%llu", (unsigned long long)n);
    if (n == 1) {
        SA_HIP(hipMemsetAsync(d_sa, 0, 4, s));
    } else {
        const Chunking ch = plan_chunks(n);
        tm.begin(SA_K_INIT);
        {
            const uint64_t grid = std::min<uint64_t>((n + kBlock * 4 - 1) / (kBlock * 4), 4096);
            hipLaunchKernelGGL(k_init_rank, dim3((uint32_t)grid), dim3(kBlock), 0, s, d_text, n, c->rank);
        }
        tm.end();
        SA_HIP(hipGetLastError());
        add_bytes(st, SA_K_INIT, 5 * n);

        uint64_t D = 256;   // manber_myers.c:94
        for (uint64_t h = 1;; h *= 2) {
            const int round = st ? st->rounds : 0;
            SA_HIP(hipEventRecord(r0, s));
            const uint32_t w = bit_width(D);          // ranks are 0..D
            const uint32_t bits = 2 * w;
            const uint32_t P = (bits + 7) / 8;
            SA_TRACE("round h=%llu D=%llu w=%u P=%u chunks=%u tpc=%u", (unsigned long long)h,
                     (unsigned long long)D, w, P, ch.chunks, ch.tiles_per_chunk);
            // index buffers: pass p writes bufs[p & 1]; make pass P-1 write d_sa
            uint32_t* vb[2];
            vb[(P - 1) & 1] = d_sa;
            vb[P & 1] = c->vals_alt;
            for (uint32_t p = 0; p < P; ++p) {
                const uint32_t shift = 8 * p;
                const uint32_t nbits = std::min<uint32_t>(8, bits - shift);
                uint64_t* ok = c->keys[p & 1];
                if (p == 0) {
                    SrcRank src{c->rank, n, h, w};
                    rc = radix_pass(c, src, ch, shift, nbits, ok, vb[0], s, tm, st, SA_K_HIST_RANK,
                                    SA_K_SCATTER_RANK, 4 * n);
                } else {
                    SrcKeys src{c->keys[(p - 1) & 1], vb[(p - 1) & 1]};
                    rc = radix_pass(c, src, ch, shift, nbits, ok, vb[p & 1], s, tm, st, SA_K_HIST_KEYS,
                                    SA_K_SCATTER_KEYS, 12 * n);
                }
                if (rc) return rc;
            }
            const uint64_t* sorted = c->keys[(P - 1) & 1];
            tm.begin(SA_K_HEADS);
            hipLaunchKernelGGL(k_heads, dim3(ch.chunks), dim3(kBlock), 0, s, sorted, ch, c->counts);
            tm.end();
            tm.begin(SA_K_HEADS_SCAN);
            hipLaunchKernelGGL(k_scan_heads, dim3(1), dim3(kBlock), 0, s, c->counts, ch.chunks, c->words);
            tm.end();
            SA_HIP(hipGetLastError());
            add_bytes(st, SA_K_HEADS, 8 * n);
            add_bytes(st, SA_K_HEADS_SCAN, 8ull * ch.chunks);
            SA_HIP(hipMemcpyAsync(c->host_words, c->words, 4, hipMemcpyDeviceToHost, s));
            SA_HIP(hipStreamSynchronize(s));
            const uint64_t Dn = c->host_words[0];
            SA_TRACE("  D'=%llu", (unsigned long long)Dn);
            const bool done = (Dn == n);
            if (!done) {
                tm.begin(SA_K_RERANK);
                hipLaunchKernelGGL(k_rerank, dim3(ch.chunks), dim3(kBlock), 0, s, sorted, (const uint32_t*)d_sa,
                                   ch, (const uint32_t*)c->counts, c->rank);
                tm.end();
                SA_HIP(hipGetLastError());
                add_bytes(st, SA_K_RERANK, 16 * n);
            }
            SA_HIP(hipEventRecord(r1, s));
            SA_HIP(hipEventSynchronize(r1));
            tm.flush();
            if (st && round < SA_MAX_ROUNDS) {
                float ms = 0.f;
                hipEventElapsedTime(&ms, r0, r1);
                st->round_ms[round] = ms;
                st->distinct[round] = Dn;
                st->passes[round] = (int32_t)P;
                // B_j = n (3 rb + 2 S (P_j + 1)), rb = 4, S = 12
                st->model_bytes += n * (3ull * 4 + 2ull * 12 * (P + 1));
            }
            if (st) st->rounds++;
            if (Dn > n || Dn == 0) return set_err(SA_E_INTERNAL, "distinct count %llu out of range",
                                                 (unsigned long long)Dn);
            if (done) break;
            if (h > n) return set_err(SA_E_INTERNAL, "doubling did not converge (h=%llu)",
                                      (unsigned long long)h);
            D = Dn;
        }
    }
    SA_HIP(hipEventRecord(r1, s));
    SA_HIP(hipEventSynchronize(r1));
    if (st) {
        float ms = 0.f;
        hipEventElapsedTime(&ms, start_all, r1);
        st->total_ms = ms;
    }
    hipEventDestroy(start_all);
    hipEventDestroy(r0);
    hipEventDestroy(r1);
    return SA_OK;
}

// ---------------------------------------------------------------------------
// O(n) checker (replaces is_valid_suffix_array, manber_myers.c:184-202)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_fill_u32(uint32_t* __restrict__ p, uint64_t n, uint32_t v) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock)
        p[i] = v;
}

// isa[sa[r]] = r; flags bit0 = index out of range, bit1 = duplicate
__global__ __launch_bounds__(kBlock) void k_check_isa(const uint32_t* __restrict__ sa, uint64_t n,
                                                      uint32_t* __restrict__ isa, uint32_t* flags) {
    uint32_t bad = 0;
    for (uint64_t r = (uint64_t)blockIdx.x * kBlock + threadIdx.x; r < n; r += (uint64_t)gridDim.x * kBlock) {
        const uint32_t x = sa[r];
        if (x >= n) { bad |= 1u; continue; }
        const uint32_t old = atomicExch(&isa[x], (uint32_t)r);
        if (old != 0xFFFFFFFFu) bad |= 2u;
    }
    if (bad) atomicOr(flags, bad);
}

// adjacent pairs: text[a] < text[b], or equal and ISA[a+1] < ISA[b+1] (ISA[n] = -1)
__global__ __launch_bounds__(kBlock) void k_check_pairs(const uint8_t* __restrict__ text,
                                                        const uint32_t* __restrict__ sa, uint64_t n,
                                                        const uint32_t* __restrict__ isa, uint32_t* flags) {
    uint32_t bad = 0;
    for (uint64_t r = (uint64_t)blockIdx.x * kBlock + threadIdx.x + 1; r < n; r += (uint64_t)gridDim.x * kBlock) {
        const uint64_t a = sa[r - 1], b = sa[r];
        const uint32_t ta = text[a], tb = text[b];
        if (ta > tb) { bad |= 4u; continue; }
        if (ta == tb) {
            const int64_t ia = (a + 1 < n) ? (int64_t)isa[a + 1] : -1;
            const int64_t ib = (b + 1 < n) ? (int64_t)isa[b + 1] : -1;
            if (!(ia < ib)) bad |= 8u;
        }
    }
    if (bad) atomicOr(flags, bad);
}

static int check_device(sa_context* c, const uint8_t* d_text, uint64_t n, const uint32_t* d_sa, hipStream_t s) {
    if (n == 0) return 1;
    if (n > 0xFFFFFFFFull) return set_err(SA_E_INVALID, "n too large");
    SA_HIP(hipSetDevice(c->device));
    int rc = ensure_capacity(c, n);
    if (rc) return rc;
    uint32_t* isa = c->rank;
    const uint32_t grid = (uint32_t)std::min<uint64_t>((n + kBlock - 1) / kBlock, 8192);
    hipLaunchKernelGGL(k_fill_u32, dim3(grid), dim3(kBlock), 0, s, isa, n, 0xFFFFFFFFu);
    SA_HIP(hipMemsetAsync(c->words + 1, 0, 4, s));
    hipLaunchKernelGGL(k_check_isa, dim3(grid), dim3(kBlock), 0, s, d_sa, n, isa, c->words + 1);
    hipLaunchKernelGGL(k_check_pairs, dim3(grid), dim3(kBlock), 0, s, d_text, d_sa, n, (const uint32_t*)isa,
                       c->words + 1);
    SA_HIP(hipGetLastError());
    SA_HIP(hipMemcpyAsync(c->host_words + 1, c->words + 1, 4, hipMemcpyDeviceToHost, s));
    SA_HIP(hipStreamSynchronize(s));
    return c->host_words[1] == 0 ? 1 : 0;
}

// ---------------------------------------------------------------------------
// seeded synthetic input on the device (SURVEY.md 8(d) splitmix64 spec), so
// benchmarks do not push gigabytes over PCIe
// ---------------------------------------------------------------------------
struct Alphabet {
    uint8_t sym[256];
};

__global__ __launch_bounds__(kBlock) void k_gen_text(uint8_t* __restrict__ out, uint64_t n, uint64_t seed,
                                                     Alphabet a, uint32_t sigma) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock) {
        uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        out[i] = a.sym[((z >> 32) * (uint64_t)sigma) >> 32];
    }
}

// process-wide context for the host-pointer entry points (lazy, locked)
static std::mutex g_mu;
static sa_context* g_ctx = nullptr;

static int global_ctx(uint64_t n, sa_context** out) {
    if (!g_ctx) {
        int rc = sa_context_create(0, n, &g_ctx);
        if (rc) return rc;
    }
    *out = g_ctx;
    return ensure_capacity(g_ctx, n);
}

}  // namespace sa

using namespace sa;

extern "C" {

const char* sa_last_error(void) { return g_err.c_str(); }

const char* sa_version(void) { return "sa_hip gfx950 " __DATE__; }

int sa_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

uint64_t sa_workspace_bytes(uint64_t max_n) { return ws_bytes(max_n); }

int sa_context_create(int device, uint64_t max_n, sa_context** out) {
    if (!out) return set_err(SA_E_INVALID, "out is NULL");
    *out = nullptr;
    int ndev = sa_device_count();
    if (ndev <= 0) return set_err(SA_E_HIP, "no HIP device visible (libsa_hip needs an MI355X)");
    if (device < 0 || device >= ndev) return set_err(SA_E_INVALID, "device %d out of range", device);
    SA_HIP(hipSetDevice(device));
    sa_context* c = new sa_context();
    c->device = device;
    if (hipMalloc(&c->hist, (size_t)kRadix * kMaxChunks * 4) != hipSuccess ||
        hipMalloc(&c->totals, kRadix * 4) != hipSuccess || hipMalloc(&c->counts, kMaxChunks * 4) != hipSuccess ||
        hipMalloc(&c->words, 64) != hipSuccess ||
        hipHostMalloc(&c->host_words, 64, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        sa_context_destroy(c);
        return set_err(SA_E_NOMEM, "context allocation failed");
    }
    for (int i = 0; i < kEvPool; ++i) {
        if (hipEventCreate(&c->ev[i]) != hipSuccess) {
            sa_context_destroy(c);
            return set_err(SA_E_HIP, "hipEventCreate failed");
        }
        c->ev_ready = i + 1;
    }
    if (max_n) {
        int rc = ensure_capacity(c, max_n);
        if (rc) {
            sa_context_destroy(c);
            return rc;
        }
    }
    *out = c;
    return SA_OK;
}

void sa_context_destroy(sa_context* c) {
    if (!c) return;
    hipSetDevice(c->device);
    free_ctx_buffers(c);
    hipFree(c->hist);
    hipFree(c->totals);
    hipFree(c->counts);
    hipFree(c->words);
    if (c->host_words) hipHostFree(c->host_words);
    for (int i = 0; i < c->ev_ready; ++i) hipEventDestroy(c->ev[i]);
    delete c;
}

int sa_build_device(sa_context* ctx, const uint8_t* d_text, uint64_t n, uint32_t* d_sa, void* stream,
                    const sa_opts* opts, sa_stats* stats) {
    if (!ctx) return set_err(SA_E_INVALID, "context is NULL");
    return build_device(ctx, d_text, n, d_sa, (hipStream_t)stream, opts, stats);
}

int sa_check_device(sa_context* ctx, const uint8_t* d_text, uint64_t n, const uint32_t* d_sa, void* stream) {
    if (!ctx) return set_err(SA_E_INVALID, "context is NULL");
    return check_device(ctx, d_text, n, d_sa, (hipStream_t)stream);
}

int sa_build_ex(const uint8_t* text, uint64_t n, void* sa_out, int sa_width, const sa_opts* opts,
                sa_stats* stats) {
    if (sa_width != 4 && sa_width != 8) return set_err(SA_E_INVALID, "sa_width must be 4 or 8");
    if (n && (!text || !sa_out)) return set_err(SA_E_INVALID, "NULL host pointer");
    if (n == 0) {
        if (stats) { std::memset(stats, 0, sizeof *stats); stats->n_kinds = SA_K_COUNT; }
        return SA_OK;
    }
    std::lock_guard<std::mutex> lk(g_mu);
    sa_context* c = nullptr;
    SA_TRACE("sa_build_ex n=%llu", (unsigned long long)n);
    int rc = global_ctx(n, &c);
    SA_TRACE("global ctx rc=%d", rc);
    if (rc) return rc;
    uint8_t* d_text = nullptr;
    uint32_t* d_sa = nullptr;
    if (hipMalloc(&d_text, align_up(n, 256)) != hipSuccess || hipMalloc(&d_sa, align_up(n, 64) * 4) != hipSuccess) {
        hipFree(d_text);
        (void)hipGetLastError();
        return set_err(SA_E_NOMEM, "device allocation of text/SA failed");
    }
    SA_TRACE("text/sa allocated");
    hipStream_t s = nullptr;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, s);
    hipError_t e = hipMemcpyAsync(d_text, text, n, hipMemcpyHostToDevice, s);
    hipEventRecord(e1, s);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    float h2d = 0.f;
    hipEventElapsedTime(&h2d, e0, e1);
    if (e == hipSuccess) {
        rc = build_device(c, d_text, n, d_sa, s, opts, stats);
    } else {
        rc = set_err(SA_E_HIP, "H2D copy failed: %s", hipGetErrorString(e));
    }
    float d2h = 0.f;
    if (rc == SA_OK) {
        hipEventRecord(e0, s);
        if (sa_width == 4) {
            e = hipMemcpyAsync(sa_out, d_sa, n * 4, hipMemcpyDeviceToHost, s);
        } else {
            std::vector<uint32_t> tmp(n);
            e = hipMemcpyAsync(tmp.data(), d_sa, n * 4, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            int64_t* o = (int64_t*)sa_out;
            for (uint64_t i = 0; i < n; ++i) o[i] = tmp[i];
        }
        hipEventRecord(e1, s);
        if (e == hipSuccess) e = hipEventSynchronize(e1);
        hipEventElapsedTime(&d2h, e0, e1);
        if (e != hipSuccess) rc = set_err(SA_E_HIP, "D2H copy failed: %s", hipGetErrorString(e));
    }
    if (stats) {
        stats->h2d_ms = h2d;
        stats->d2h_ms = d2h;
    }
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    hipFree(d_text);
    hipFree(d_sa);
    return rc;
}

int sa_generate_text_device(uint8_t* d_out, uint64_t n, uint64_t seed, const uint8_t* alphabet, uint32_t sigma,
                            void* stream) {
    if (n == 0) return SA_OK;
    if (!d_out || !alphabet || sigma == 0 || sigma > 256) return set_err(SA_E_INVALID, "bad generator arguments");
    Alphabet a;
    std::memset(a.sym, 0, sizeof a.sym);
    std::memcpy(a.sym, alphabet, sigma);
    const uint32_t grid = (uint32_t)std::min<uint64_t>((n + kBlock - 1) / kBlock, 16384);
    hipLaunchKernelGGL(k_gen_text, dim3(grid), dim3(kBlock), 0, (hipStream_t)stream, d_out, n, seed, a, sigma);
    SA_HIP(hipGetLastError());
    return SA_OK;
}

int sa_check(const uint8_t* text, uint64_t n, const void* sa, int sa_width) {
    if (sa_width != 4 && sa_width != 8) return set_err(SA_E_INVALID, "sa_width must be 4 or 8");
    if (n == 0) return 1;
    if (!text || !sa) return set_err(SA_E_INVALID, "NULL host pointer");
    if (n > 0xFFFFFFFFull) return set_err(SA_E_INVALID, "n too large");
    std::vector<uint32_t> narrow;
    const void* src = sa;
    if (sa_width == 8) {
        narrow.resize(n);
        const int64_t* w = (const int64_t*)sa;
        for (uint64_t i = 0; i < n; ++i) {
            if (w[i] < 0 || (uint64_t)w[i] >= n) return 0;
            narrow[i] = (uint32_t)w[i];
        }
        src = narrow.data();
    }
    std::lock_guard<std::mutex> lk(g_mu);
    sa_context* c = nullptr;
    int rc = global_ctx(n, &c);
    if (rc) return rc;
    uint8_t* d_text = nullptr;
    uint32_t* d_sa = nullptr;
    if (hipMalloc(&d_text, align_up(n, 256)) != hipSuccess || hipMalloc(&d_sa, align_up(n, 64) * 4) != hipSuccess) {
        hipFree(d_text);
        (void)hipGetLastError();
        return set_err(SA_E_NOMEM, "device allocation failed");
    }
    rc = SA_OK;
    if (hipMemcpy(d_text, text, n, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_sa, src, n * 4, hipMemcpyHostToDevice) != hipSuccess)
        rc = set_err(SA_E_HIP, "H2D copy failed");
    if (rc == SA_OK) rc = check_device(c, d_text, n, d_sa, nullptr);
    hipFree(d_text);
    hipFree(d_sa);
    return rc;
}

}  // extern "C"
