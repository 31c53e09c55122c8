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
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/sa_hip.h"

// alphabet kernel workgroups (overridable for A/B runs)
#ifndef SA_ALPHA_GRID
#define SA_ALPHA_GRID 2048
#endif

#include "sa_bucket.h"
#include "sa_check.h"
#include "sa_kernels.h"
#include "sa_lcp.h"
#include "sa_limits.h"
#include "sa_onesweep.h"
#include "sa_permute.h"
#include "sa_pivot.h"
#include "sa_split.h"
#include "sa_lsd.h"

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

// Every host wait of the library goes through these two (a stream sync, or
// a blocking copy): sa_host_syncs() reports their count, so a driver can
// show how many times a build stops the host (bench.py host_syncs_per_build).
static std::atomic<uint64_t> g_host_syncs{0};
static hipError_t host_sync(hipStream_t s) {
    g_host_syncs.fetch_add(1, std::memory_order_relaxed);
    return hipStreamSynchronize(s);
}
static hipError_t host_memcpy(void* dst, const void* src, size_t bytes, hipMemcpyKind kind) {
    g_host_syncs.fetch_add(1, std::memory_order_relaxed);
    return hipMemcpy(dst, src, bytes, kind);
}

// propagate a non-zero status (variadic: template arguments carry commas)
#define SA_TRY(...)                      \
    do {                                 \
        const int rc_ = (__VA_ARGS__);   \
        if (rc_) return rc_;             \
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

// chunks of the chunked (tile-sequential) kernels: 4096 workgroups keep 16
// per CU in flight on the 256 CUs
#ifndef SA_MAX_CHUNKS
#define SA_MAX_CHUNKS 4096   // 16384 cut degenerate k_seg_write 317 -> 298 ms
#endif
constexpr uint32_t kMaxChunks = SA_MAX_CHUNKS;
// the one-workgroup chunk scans (k_seg_scan, k_scan_heads, k_scan_chunk_max)
// loop over blocks with a carry; the scratch arrays are sized by kMaxChunks
static_assert(kMaxChunks >= 1 && kMaxChunks <= (1u << 20), "chunk scratch sized for at most 2^20 chunks");
// sparse round-1 ranks when at most n / kSparseDiv suffixes stay unsorted
constexpr uint64_t kSparseDiv = 8;
constexpr int kEvPool = 256;
constexpr int kRoundEv = SA_MAX_ROUNDS + 1;   // round boundary events (Timer::round_mark)

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

namespace sa { struct DistState; }

struct sa_context {
    int device = 0;
    uint64_t cap = 0;      // rank / keys / vals_alt capacity (symbols)
    uint64_t cap_pad = 0;  // keys[0] / vals_alt capacity in elements (>= cap; padded first-pass segments)
    uint64_t ucap = 0;     // unsorted-set buffers capacity
    uint32_t* rank = nullptr;
    uint64_t* keys[2] = {nullptr, nullptr};
    uint32_t* vals_alt = nullptr;
    uint32_t* vals_u = nullptr;                 // sorted idx of an unsorted-set round
    uint32_t* u_pos[2] = {nullptr, nullptr};    // compacted unsorted set, ping-pong
    uint32_t* u_idx[2] = {nullptr, nullptr};
    uint32_t* u_g[2] = {nullptr, nullptr};
    uint32_t* u_gs[2] = {nullptr, nullptr};     // each set's group starts (pivot rounds; allocated at the first)
    uint64_t gscap = 0;
    uint64_t* keys_u = nullptr;                 // third key buffer (unsorted-set rounds)
    uint64_t kucap = 0;                         // keys_u capacity (items): ucap + the XQ regions' slack
    uint32_t* segx = nullptr;                   // second bucket pass, per-XCD queues (sa_split.h SegXq) + tables
    uint64_t segx_words = 0;
    uint32_t* os = nullptr;                     // onesweep ghist / digit bases / tickets
    uint32_t* lsd = nullptr;                    // k_lsd ghist [8][1024] | bases [8][1024] | tickets [8]
    uint32_t* lsdx = nullptr;                   // XQ k_lsd: per-queue counts [passes][8][1024] | bases [8][1024] | tickets
    uint32_t* segw = nullptr;                   // second bucket pass: per-segment cursors / bases / flags
    uint64_t* states = nullptr;                 // onesweep tile states [tiles][256]
    uint32_t epoch = 0;                         // onesweep state tag of the last pass
    int radix = 0;                              // 0 onesweep, 1 reduce-then-scan
    int cus = 256;                              // compute units (persistent grids)
    uint32_t* member = nullptr;                 // bitmap of round-1 unsorted positions
    uint32_t* hist = nullptr;      // 256 * kMaxChunks
    uint32_t* totals = nullptr;    // 256
    uint32_t* counts = nullptr;    // 4 * kMaxChunks (heads, u, uheads, last)
    uint32_t* words = nullptr;     // [0..2] = D, m, G; [3] = check error flags
    uint32_t* alpha = nullptr;     // 256 byte counts
    uint16_t* code = nullptr;      // 256 byte -> dense code 1..sigma
    uint32_t* host_words = nullptr;  // pinned (4096 words): 64 words, 256 counts, 128 words of codes at 320, the text tail (64 B) at 2048,
                                     // per-rank counts of the range-partitioned build at 1024
    hipEvent_t ev[sa::kEvPool + sa::kRoundEv];   // Timer pairs, then the round boundaries
    int ev_ready = 0;
    sa::DistState* dist = nullptr;   // range-partitioned build state (sa_dist.h)
    // sa_opts debug / tune fields of the current build (sa_build_device's
    // opts, or sa_context_set_debug for the sa_dist_* phases)
    uint32_t dbg = 0;
    int32_t span_extra = 0;
    int32_t tune = 0;
    bool dna = false;   // the text's alphabet is exactly {A, C, G, T} (k_split_text<.., DNA>)
    bool samples_pending = false;   // round 1 wrote no key1 samples (SegOut::samples = 0)
};

namespace sa {

// keys[0] / vals_alt elements for the padded first-pass segments of the
// bucketed round (sa_round1.h kPadMinN..kPadMaxN; their bound sums to < 1.1 n)
static uint64_t pad_capacity(uint64_t n) { return n + n / 8 + (1ull << 22); }

// keys[0] / vals_alt capacity (elements) of a context for n symbols
static uint64_t pad_elems(uint64_t n) {
    const uint64_t m = align_up(std::max<uint64_t>(n, 1), 64);
    return (n >= (1ull << 26) && n <= (1ull << 31)) ? align_up(pad_capacity(n), 64) : m;
}

// tile states for the widest digit (the bucketed first round's high pass
// uses up to 10 bits)
constexpr uint64_t kMaxRadix = 1024;
static uint64_t tile_states_bytes(uint64_t n) { return ((n + kTile - 1) / kTile + 1) * kMaxRadix * 8; }

// Device memory a context holds for n symbols: rank + 2 key + 1 index buffer
// (the reference schedule; keys[0] and the index buffer padded, pad_elems),
// plus 7 u32 arrays for the unsorted set (packed), keys_u with the per-XCD
// regions' slack (ensure_u_capacity), the group starts of pivot rounds
// (ensure_gs, 2 x (n/2 + 64) words) and the second pass's queue workspace
// (sa_round1.h: xq_words(1024) + 1032 + 2 x 8 x 2^19 bucket-table words at
// most) and the single-pass radix tile states.
static uint64_t ws_bytes(uint64_t n) {
    const uint64_t m = align_up(std::max<uint64_t>(n, 1), 64);
    const uint64_t ku_slack = n >= (1ull << 26) ? n / 16 + 8ull * 1024 * kXqSlack + 64 : 0;
    const uint64_t gs = 2 * (n / 2 + 64) * 4;
    const uint64_t segx = (xq_words(1024) + 1032 + 2ull * kXq * (1ull << 19)) * 4;
    return m * 4 + 2 * m * 8 + m * 4 + (pad_elems(n) - m) * 12 + 7 * m * 4 + (m + ku_slack) * 8 + m / 8 + gs +
           segx + tile_states_bytes(n) + (uint64_t)kRadix * kMaxChunks * 4 + 8192;
}

static void free_ctx_buffers(sa_context* c) {
    hipFree(c->rank);
    hipFree(c->keys[0]);
    hipFree(c->keys[1]);
    hipFree(c->vals_alt);
    hipFree(c->states);
    c->rank = nullptr;
    c->keys[0] = c->keys[1] = nullptr;
    c->vals_alt = nullptr;
    c->states = nullptr;
    c->cap = 0;
    c->cap_pad = 0;
}

static void free_u_buffers(sa_context* c) {
    hipFree(c->vals_u);
    hipFree(c->keys_u);
    hipFree(c->member);
    c->vals_u = nullptr;
    c->keys_u = nullptr;
    c->member = nullptr;
    for (int i = 0; i < 2; ++i) {
        hipFree(c->u_pos[i]);
        hipFree(c->u_idx[i]);
        hipFree(c->u_g[i]);
        hipFree(c->u_gs[i]);
        c->u_pos[i] = c->u_idx[i] = c->u_g[i] = c->u_gs[i] = nullptr;
    }
    c->gscap = 0;
    c->ucap = 0;
    c->kucap = 0;
}

// sa_opts debug / tune fields -> the context (NULL: production defaults)
static void set_debug(sa_context* c, const sa_opts* o) {
    c->dbg = o ? o->debug : 0u;
    c->span_extra = o ? o->span_extra : 0;
    c->tune = o ? o->tune : 0;
}

static int ensure_capacity(sa_context* c, uint64_t n) {
    if (n <= c->cap && c->rank) return SA_OK;
    SA_HIP(hipSetDevice(c->device));
    free_ctx_buffers(c);
    const uint64_t m = align_up(std::max<uint64_t>(n, 1), 64);
    // padded segments from 2^26 up to 2^31 suffixes (the bucketed round's
    // one-GPU maximum)
    const uint64_t mp = pad_elems(n);
    if (hipMalloc(&c->rank, m * 4) != hipSuccess || hipMalloc(&c->keys[0], mp * 8) != hipSuccess ||
        hipMalloc(&c->keys[1], m * 8) != hipSuccess || hipMalloc(&c->vals_alt, mp * 4) != hipSuccess ||
        hipMalloc(&c->states, tile_states_bytes(n)) != hipSuccess ||
        hipMemset(c->states, 0, tile_states_bytes(n)) != hipSuccess) {
        free_ctx_buffers(c);
        (void)hipGetLastError();
        return set_err(SA_E_NOMEM, "device allocation of %.2f GiB workspace failed",
                       (double)ws_bytes(n) / (1ull << 30));
    }
    c->cap = n;
    c->cap_pad = mp;
    SA_TRACE("workspace: rank %p keys0 %p keys1 %p vals_alt %p", (void*)c->rank, (void*)c->keys[0], (void*)c->keys[1],
             (void*)c->vals_alt);
    return SA_OK;
}

static int ensure_u_capacity(sa_context* c, uint64_t n) {
    if (n <= c->ucap && c->vals_u) return SA_OK;
    SA_HIP(hipSetDevice(c->device));
    free_u_buffers(c);
    const uint64_t m = align_up(std::max<uint64_t>(n, 1), 64) * 4;
    // keys_u also holds the second bucket pass's per-XCD regions (sa_split.h
    // SegXq): n items plus each (queue, digit) sub-region's slack, at most
    // n / 16 + 8 * 1024 * kXqSlack items (padded first-pass sizes only)
    const uint64_t ku = align_up(std::max<uint64_t>(n, 1), 64) +
                        (n >= (1ull << 26) ? n / 16 + 8ull * 1024 * kXqSlack + 64 : 0);
    bool ok = hipMalloc(&c->vals_u, m) == hipSuccess && hipMalloc(&c->keys_u, 8 * ku) == hipSuccess &&
              hipMalloc(&c->member, align_up(n, 1024) / 8) == hipSuccess;
    for (int i = 0; i < 2 && ok; ++i)
        ok = hipMalloc(&c->u_pos[i], m) == hipSuccess && hipMalloc(&c->u_idx[i], m) == hipSuccess &&
             hipMalloc(&c->u_g[i], m) == hipSuccess;
    if (!ok) {
        free_u_buffers(c);
        (void)hipGetLastError();
        return set_err(SA_E_NOMEM, "device allocation of the unsorted-set buffers failed");
    }
    c->ucap = n;
    c->kucap = ku;
    SA_TRACE("unsorted-set buffers: vals_u %p keys_u %p", (void*)c->vals_u, (void*)c->keys_u);
    return SA_OK;
}

// each unsorted set's group starts (pivot rounds, sa_pivot.h MODE 1): G <=
// m / 2 <= n / 2 words per set, allocated when a build first takes a pivot
// round (range builds never do)
static int ensure_gs(sa_context* c, uint64_t n) {
    if (n <= c->gscap && c->u_gs[0]) return SA_OK;
    for (int i = 0; i < 2; ++i) {
        hipFree(c->u_gs[i]);
        c->u_gs[i] = nullptr;
    }
    c->gscap = 0;
    const uint64_t w = n / 2 + 64;
    for (int i = 0; i < 2; ++i)
        if (hipMalloc(&c->u_gs[i], w * 4) != hipSuccess) {
            (void)hipGetLastError();
            for (int k = 0; k < 2; ++k) {
                hipFree(c->u_gs[k]);
                c->u_gs[k] = nullptr;
            }
            return set_err(SA_E_NOMEM, "group-start buffers (%llu words)", (unsigned long long)w);
        }
    c->gscap = n;
    return SA_OK;
}

// ensure_gs for a path that has an alternative: false (the HIP error and
// the message cleared) when the buffers cannot be allocated
static bool gs_available(sa_context* c, uint64_t n) {
    if (ensure_gs(c, n) == SA_OK) return true;
    (void)hipGetLastError();
    g_err.clear();
    SA_TRACE("group-start buffers unavailable: pivot rounds without tied blocks");
    return false;
}

// set i's group-start buffer when it holds an n-suffix build's groups
static uint32_t* gs_buf(const sa_context* c, uint64_t n, int i) { return n <= c->gscap ? c->u_gs[i] : nullptr; }

// Per-launch HIP-event timing, enabled by sa_opts.profile.
struct Timer {
    sa_context* c;
    hipStream_t s;
    bool on;
    sa_stats* st;
    int used = 0;
    int kind[kEvPool / 2];
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
    // round boundaries: one event before the first round and one after each,
    // read when the build has finished (round_times), so no round waits for
    // the GPU to drain before the next one is launched
    int nr = 0;
    uint64_t mark_bytes[kRoundEv] = {};   // the stats' algorithmic bytes at each boundary
    void round_mark() {
        if (nr < kRoundEv) {
            hipEventRecord(c->ev[kEvPool + nr], s);
            uint64_t b = 0;
            if (st)
                for (int k = 0; k < SA_K_COUNT; ++k) b += st->kern_bytes[k];
            mark_bytes[nr] = b;
        }
        ++nr;
    }
    void round_times() {
        const int last = std::min(nr, kRoundEv) - 1;
        if (!st || last < 1) return;
        hipEventSynchronize(c->ev[kEvPool + last]);
        for (int r = 0; r < last && r < st->rounds; ++r) {
            float ms = 0.f;
            hipEventElapsedTime(&ms, c->ev[kEvPool + r], c->ev[kEvPool + r + 1]);
            st->round_ms[r] = ms;
            st->round_bytes[r] = mark_bytes[r + 1] - mark_bytes[r];
        }
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

// owned HIP events (destroyed on every return path)
struct Events {
    hipEvent_t e[3] = {nullptr, nullptr, nullptr};
    int make() {
        for (auto& x : e)
            if (hipEventCreate(&x) != hipSuccess) return set_err(SA_E_HIP, "hipEventCreate failed");
        return SA_OK;
    }
    ~Events() {
        for (auto& x : e)
            if (x) hipEventDestroy(x);
    }
};

static float elapsed(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

static void add_bytes(sa_stats* st, int kind, uint64_t b) {
    if (st) st->kern_bytes[kind] += b;
}

// One LSD radix pass over bits [shift, shift + nbits).
template <class Src>
static int radix_pass(sa_context* c, const Src& src, const Chunking& ch, uint32_t shift, uint32_t nbits,
                      uint64_t* out_keys, uint32_t* out_vals, hipStream_t s, Timer& tm, sa_stats* st,
                      int kind_hist, int kind_scatter, uint64_t in_bytes, bool hist_ready = false) {
    const uint32_t mask = (1u << nbits) - 1u;
    if (!hist_ready) {
        tm.begin(kind_hist);
        hipLaunchKernelGGL(k_hist<Src>, dim3(ch.chunks), dim3(kBlock), 0, s, src, ch, shift, mask, c->hist);
        tm.end();
        add_bytes(st, kind_hist, in_bytes);
    }
    tm.begin(SA_K_SCAN);
    hipLaunchKernelGGL(k_scan_rows, dim3(kRadix), dim3(kBlock), 0, s, c->hist, ch.chunks, c->totals);
    tm.end();
    tm.begin(kind_scatter);
    hipLaunchKernelGGL(k_scatter<Src>, dim3(ch.chunks), dim3(kBlock), 0, s, src, ch, shift, nbits,
                       (const uint32_t*)c->hist, (const uint32_t*)c->totals, out_keys, out_vals);
    tm.end();
    SA_HIP(hipGetLastError());
    add_bytes(st, SA_K_SCAN, 2ull * 4 * kRadix * ch.chunks);
    add_bytes(st, kind_scatter, in_bytes + 12ull * ch.n);
    return SA_OK;
}

// single-pass (onesweep) scratch: ghist[8][256] | base[8][256] | tickets[8]
static uint32_t* os_ghist(sa_context* c) { return c->os; }
static uint32_t* os_base(sa_context* c) { return c->os + kMaxPasses * kRadix; }
static uint32_t* os_tickets(sa_context* c) { return c->os + 2 * kMaxPasses * kRadix; }

// zero the global histograms and tile tickets of the next sort
static int onesweep_prepare(sa_context* c, hipStream_t s) {
    SA_HIP(hipMemsetAsync(c->os, 0, (2 * kMaxPasses * kRadix + kMaxPasses) * 4, s));
    return SA_OK;
}

static uint32_t next_epoch(sa_context* c, hipStream_t s) {
    if (++c->epoch > kEpochMask) {
        hipMemsetAsync(c->states, 0, tile_states_bytes(c->cap), s);
        c->epoch = 1;
    }
    return c->epoch;
}

template <class Src, int RBITS = 8>
static void onesweep_pass(sa_context* c, const Src& src, uint64_t n, uint32_t shift, uint32_t nbits,
                          const uint32_t* base, uint32_t* ticket, uint64_t* out_keys, uint32_t* out_vals,
                          hipStream_t s) {
    const uint64_t tiles = (n + kTile - 1) / kTile;
    const uint32_t epoch = next_epoch(c, s);
    // 1024 x 4: 16 waves per tile, 2 workgroups (32 waves) per CU -- the
    // fastest shape in microbench.hip (r01: 10.4 ms per 2^30-pair pass)
    static_assert(kOsBlock * kOsItems == kTile, "tile states are sized for kTile");
    hipLaunchKernelGGL((k_onesweep<Src, kOsBlock, kOsItems, RBITS>), dim3((uint32_t)tiles), dim3(kOsBlock), 0, s, src,
                       n, shift, nbits, base, c->states, ticket, epoch, out_keys, out_vals, c->words + 4);
}

// Stable LSD sort of ch.n (key, idx) pairs over key bits [0, bits): the first
// pass generates pairs from `first`, later passes read the ping-pong buffers.
// The sorted idx land in vals_final; *sorted_keys = the sorted key buffer.
// hist0_ready: the first source's histograms are already computed (per chunk
// for the reduce-then-scan sort; global, after onesweep_prepare, otherwise).
template <class Src>
static int radix_sort(sa_context* c, const Src& first, uint64_t first_bytes, const Chunking& ch, uint32_t bits,
                      uint32_t* vals_final, uint32_t* vals_other, uint64_t* kb0, uint64_t* kb1, hipStream_t s,
                      Timer& tm, sa_stats* st, uint64_t** sorted_keys, uint32_t* passes, bool hist0_ready = false,
                      bool usort = false) {
    const uint32_t P = (bits + 7) / 8;
    if (P > kMaxPasses) return set_err(SA_E_INTERNAL, "%u radix passes", P);
    // an unsorted-set sort (later rounds, few suffixes) is accounted apart so
    // the per-kind averages of the full-n passes stay per-launch comparable
    const int k_hist = usort ? SA_K_SORT_U : SA_K_HIST_FIRST;
    const int k_first = usort ? SA_K_SORT_U : SA_K_SCATTER_FIRST;
    const int k_keys = usort ? SA_K_SORT_U : SA_K_SCATTER_KEYS;
    if (c->radix == 0) {
        const uint64_t n = ch.n;
        uint32_t* vb[2];
        vb[(P - 1) & 1] = vals_final;
        vb[P & 1] = vals_other;
        uint64_t* kb[2] = {kb0, kb1};
        if (!hist0_ready) {
            int rc = onesweep_prepare(c, s);
            if (rc) return rc;
            tm.begin(k_hist);
            const uint32_t grid = (uint32_t)std::min<uint64_t>((n + kBlock - 1) / kBlock, 2048);
            hipLaunchKernelGGL(k_global_hist<Src>, dim3(grid), dim3(kBlock), 0, s, first, n, P, os_ghist(c));
            tm.end();
            add_bytes(st, k_hist, first_bytes);
        }
        tm.begin(SA_K_SCAN);
        hipLaunchKernelGGL(k_digit_base, dim3(P), dim3(kBlock), 0, s, (const uint32_t*)os_ghist(c), os_base(c));
        tm.end();
        for (uint32_t p = 0; p < P; ++p) {
            const uint32_t shift = 8 * p;
            const uint32_t nbits = std::min<uint32_t>(8, bits - shift);
            if (p == 0) {
                tm.begin(k_first);
                onesweep_pass(c, first, n, shift, nbits, os_base(c), os_tickets(c), kb[0], vb[0], s);
                tm.end();
                add_bytes(st, k_first, first_bytes + 12 * n);
            } else {
                SrcKeys src{kb[(p - 1) & 1], vb[(p - 1) & 1]};
                tm.begin(k_keys);
                onesweep_pass(c, src, n, shift, nbits, os_base(c) + p * kRadix, os_tickets(c) + p, kb[p & 1],
                              vb[p & 1], s);
                tm.end();
                add_bytes(st, k_keys, 24 * n);
            }
        }
        SA_HIP(hipGetLastError());
        *sorted_keys = kb[(P - 1) & 1];
        *passes = P;
        return SA_OK;
    }
    uint32_t* vb[2];
    vb[(P - 1) & 1] = vals_final;
    vb[P & 1] = vals_other;
    uint64_t* kb[2] = {kb0, kb1};
    for (uint32_t p = 0; p < P; ++p) {
        const uint32_t shift = 8 * p;
        const uint32_t nbits = std::min<uint32_t>(8, bits - shift);
        int rc;
        if (p == 0) {
            rc = radix_pass(c, first, ch, shift, nbits, kb[0], vb[0], s, tm, st, k_hist, k_first, first_bytes,
                            hist0_ready);
        } else {
            SrcKeys src{kb[(p - 1) & 1], vb[(p - 1) & 1]};
            rc = radix_pass(c, src, ch, shift, nbits, kb[p & 1], vb[p & 1], s, tm, st,
                            usort ? SA_K_SORT_U : SA_K_HIST_KEYS, k_keys, 12 * ch.n);
        }
        if (rc) return rc;
    }
    *sorted_keys = kb[(P - 1) & 1];
    *passes = P;
    return SA_OK;
}

#include "sa_round1.h"

static void record_round(sa_stats* st, float ms, uint64_t D, uint32_t P, uint64_t sorted_n, uint64_t h) {
    if (!st) return;
    const int r = st->rounds;
    if (r < SA_MAX_ROUNDS) {
        st->round_ms[r] = ms;
        st->distinct[r] = D;
        st->passes[r] = (int32_t)P;
        st->sorted_n[r] = sorted_n;
        st->prefix_len[r] = h;
    }
    // B_j = n_j (3 rb + 2 S (P_j + 1)), rb = 4, S = 12
    st->model_bytes += sorted_n * (3ull * 4 + 2ull * 12 * (P + 1));
    st->rounds++;
}

// ---------------------------------------------------------------------------
// reference schedule: manber_myers.c:88-125 round for round
// ---------------------------------------------------------------------------
// the re-rank as a permutation (sa_permute.h) from this many suffixes; below
// it rank[] stays inside the L2s and one random scatter (k_rerank) is cheaper
// (SA_DEBUG_PERM_ALWAYS: from any n, for tests at small n)
constexpr int kPermErrWord = 13;
static uint64_t perm_min_n(const sa_context* c) { return (c->dbg & SA_DEBUG_PERM_ALWAYS) ? 1ull : (1ull << 22); }

static PermPlan plan_perm(uint64_t n) {
    PermPlan p;
    const uint32_t lg = bit_width(n > 1 ? n - 1 : 1);   // ceil(log2 n)
    p.s2 = kPermSub;
    p.s1 = std::max<uint32_t>(p.s2, lg > 8 ? lg - 8 : 0);
    p.nb1 = (uint32_t)((n + (1ull << p.s1) - 1) >> p.s1);
    p.nsub = 1u << (p.s1 - p.s2);
    p.tpb = (uint32_t)(((1ull << p.s1) + kPermBlock * kPermItems - 1) / (kPermBlock * kPermItems));
    return p;
}

// rank[idx[p]] = dense rank of sorted position p, through the two key
// buffers (the sorted keys are read by the first step and then free)
// first-level tiles of the permutation and their head offsets (k_tile_heads)
constexpr uint64_t kPermTile = (uint64_t)kPermBlock * kPermItems;
static_assert((kPermTile & (kPermTile - 1)) == 0, "power-of-two first-level tiles");
static uint32_t* perm_tile_off(sa_context* c) { return c->hist + ((uint64_t)kRadix * kMaxChunks) / 2; }
// tickets of the persistent permutation kernels: below the re-rank's tile offsets in hist
static uint32_t* perm_tickets(sa_context* c) { return c->hist + ((uint64_t)kRadix * kMaxChunks) / 2 - 64; }

static int rerank_permute(sa_context* c, uint64_t* sorted, const uint32_t* d_sa, const Chunking& ch,
                          hipStream_t s, Timer& tm, sa_stats* st, uint32_t kshift = 0, NextHist nh = NextHist{}) {
    const uint64_t n = ch.n;
    const PermPlan p = plan_perm(n);
    const uint64_t half = (uint64_t)kRadix * kMaxChunks / 2;   // cursors below, tile offsets above
    if (p.nb1 > 256 || p.nsub > kPermMaxSub || 256ull + (uint64_t)p.nb1 * p.nsub > half ||
        (n + kPermTile - 1) / kPermTile > half)
        return set_err(SA_E_INTERNAL, "permutation plan out of range (n=%llu)", (unsigned long long)n);
    uint64_t* other = sorted == c->keys[0] ? c->keys[1] : c->keys[0];
    uint32_t* cur1 = c->hist;          // the chunk histograms are free after the sort
    uint32_t* cur2 = c->hist + 256;
    SA_HIP(hipMemsetAsync(c->hist, 0, (256ull + (uint64_t)p.nb1 * p.nsub) * 4, s));
    tm.begin(SA_K_RERANK);
    const uint32_t tiles = (uint32_t)((n + kPermTile - 1) / kPermTile);
    const uint32_t* toff = perm_tile_off(c);
    if (kshift)   // packed (key << kshift | idx) items
        hipLaunchKernelGGL((k_perm_rank<kPermBlock, kPermItems, true>), dim3(tiles), dim3(kPermBlock), 0, s,
                           (const uint64_t*)sorted, d_sa, n, toff, p.s1, kshift, cur1, other);
    else
        hipLaunchKernelGGL((k_perm_rank<kPermBlock, kPermItems, false>), dim3(tiles), dim3(kPermBlock), 0, s,
                           (const uint64_t*)sorted, d_sa, n, toff, p.s1, 0u, cur1, other);
    const uint64_t* placed = other;
    if (p.s1 > p.s2) {
        if ((((uint32_t)c->tune >> 24) & 0xFu) == 1u) {   // A/B: the persistent prefetching split
            uint32_t* tk = perm_tickets(c);
            SA_HIP(hipMemsetAsync(tk, 0, 8 * 4, s));
            hipLaunchKernelGGL((k_split_p<kPermBlock, kPermItems>), dim3(2 * (uint32_t)c->cus), dim3(kPermBlock), 0, s,
                               (const uint64_t*)other, n, p.s1, p.s2, p.nb1, 1u, (uint64_t)0, p.tpb,
                               (const uint32_t*)nullptr, 0u, cur2, sorted, tk);
        } else {
            hipLaunchKernelGGL((k_perm_split<kPermBlock, kPermItems>), dim3((p.nb1 + 7) / 8 * 8 * p.tpb),
                               dim3(kPermBlock), 0, s, (const uint64_t*)other, n, p.s1, p.s2, p.tpb, cur2, sorted);
        }
        placed = sorted;
    }
    if (nh.out) {   // the next round's first-digit counts too (persistent: one count flush per workgroup)
        SA_HIP(hipMemsetAsync(nh.out, 0, 8 * kLsdMaxRadix * 4, s));
        const uint64_t nsub = (n + (1ull << kPermSub) - 1) >> kPermSub;
        const uint64_t g = std::min<uint64_t>(nsub, 2ull * (uint64_t)c->cus);   // two workgroups per CU
        const uint32_t spb = (uint32_t)((nsub + g - 1) / g);
        hipLaunchKernelGGL((k_perm_place<kPermBlock, true>), dim3((uint32_t)((nsub + spb - 1) / spb)),
                           dim3(kPermBlock), 0, s, placed, n, c->rank, c->words + kPermErrWord, nh, spb);
    } else {
        hipLaunchKernelGGL((k_perm_place<kPermBlock>), dim3((uint32_t)((n + (1ull << kPermSub) - 1) >> kPermSub)),
                           dim3(kPermBlock), 0, s, placed, n, c->rank, c->words + kPermErrWord);
    }
    tm.end();
    SA_HIP(hipGetLastError());
    add_bytes(st, SA_K_RERANK, (p.s1 > p.s2 ? 48ull : 32ull) * n - (kshift ? 4ull * n : 0ull));
    return SA_OK;
}

// ---------------------------------------------------------------------------
// the reference schedule's LSD sort (sa_lsd.h)
// ---------------------------------------------------------------------------
static uint32_t* lsd_ghist(sa_context* c) { return c->lsd; }
static uint32_t* lsd_base(sa_context* c) { return c->lsd + kMaxPasses * kLsdMaxRadix; }
static uint32_t* lsd_tickets(sa_context* c) { return c->lsd + 2 * kMaxPasses * kLsdMaxRadix; }

// widest digit of the plan (sa_opts.tune bits 0-7 = 8 restores 8-bit
// digits, A/B)
static uint32_t lsd_max_bits(const sa_context* c) {
    const uint32_t b = (uint32_t)c->tune & 0xFFu;
    return b ? std::min<uint32_t>(10, std::max<uint32_t>(8, b)) : 10u;
}

// B key bits above bit `base`: the pass count and widths of least relative
// cost, a pass of 9 / 10 bits costing ~1.2 / 1.45 of an 8-bit one (longer
// match-any, shorter digit runs per tile)
static LsdPlan lsd_plan(uint32_t B, uint32_t base, uint32_t maxb) {
    auto cost = [](uint32_t w) { return w <= 8 ? 1.0 : w == 9 ? 1.2 : 1.45; };
    LsdPlan pl{};
    double best = 1e30;
    for (uint32_t p = std::max<uint32_t>(1, (B + maxb - 1) / maxb); p <= std::max<uint32_t>(1, (B + 7) / 8); ++p) {
        double cst = 0;
        for (uint32_t i = 0; i < p; ++i) cst += cost(B / p + (i < B % p ? 1u : 0u));
        if (cst < best - 1e-9) {
            best = cst;
            pl.P = p;
        }
    }
    uint32_t sh = base;
    for (uint32_t i = 0; i < pl.P; ++i) {
        pl.bits[i] = std::max<uint32_t>(1, B / pl.P + (i < B % pl.P ? 1u : 0u));
        pl.shift[i] = sh;
        sh += pl.bits[i];
    }
    return pl;
}

// resident workgroups per CU of a persistent kernel (a property of the code
// object, the same on every gfx950 device; the grid is this times the
// launching context's CU count)
template <class K>
static int blocks_per_cu(K kernel, int block) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, block, 0) != hipSuccess || nb < 1) nb = 1;
    return nb;
}

// XQ (sa_lsd.h): per-XCD queues of tiles; base = qbase[8][1024], ticket =
// the pass's 8 queue tickets, next_hist = the next pass's per-queue counts;
// the grid is whole XCDs (every queue served)
template <class Src, bool PACKED, bool XQ = false>
static int lsd_pass(sa_context* c, const Src& src, uint64_t n, uint32_t shift, uint32_t nbits, const uint32_t* base,
                     uint32_t* ticket, uint64_t* ok, uint32_t* ov, hipStream_t s, uint32_t nshift, uint32_t nnbits,
                     uint32_t* next_hist, QDiv qd = QDiv{}, uint32_t tpq = 0) {
    const uint32_t epoch = next_epoch(c, s);
    uint64_t tiles = 0;
    unsigned long long* prof = reinterpret_cast<unsigned long long*>(lsd_tickets(c) + kMaxPasses);
    if (SA_LSD_PROF) hipMemsetAsync(prof, 0, 5 * 8, s);
#define SA_LSD_LAUNCH(RB)                                                                                   \
    do {                                                                                                    \
        auto kern = k_lsd<Src, RB, PACKED, XQ>;                                                             \
        constexpr int B = lsd_block<PACKED, RB, XQ>();                                                      \
        constexpr uint64_t T = (uint64_t)B * lsd_items<PACKED, RB, XQ>();                                   \
        tiles = (n + T - 1) / T;                                                                            \
        static std::atomic<int> per_cu{0};                                                                  \
        if (!per_cu.load(std::memory_order_relaxed)) per_cu.store(blocks_per_cu(kern, B));                  \
        const uint64_t grid = (uint64_t)c->cus * (uint64_t)per_cu.load(std::memory_order_relaxed);          \
        hipLaunchKernelGGL(kern, dim3((uint32_t)(XQ ? grid : std::min<uint64_t>(tiles, grid))), dim3(B), 0, s, \
                           src, n, shift, nbits, base, c->states, ticket, epoch, ok, ov, c->words + 4, prof,   \
                           nshift, nnbits, next_hist, qd, tpq);                                            \
    } while (0)
    if (nbits <= 8) SA_LSD_LAUNCH(8);
    else if (nbits == 9) SA_LSD_LAUNCH(9);
    else if constexpr (PACKED || !XQ) SA_LSD_LAUNCH(10);
    else   // unpacked XQ passes take <= 9 bits (lsd_xq_ok): a wider one would write nothing
        return set_err(SA_E_INTERNAL, "unpacked per-XCD LSD pass of %u bits", nbits);
#undef SA_LSD_LAUNCH
    if (SA_LSD_PROF) {
        unsigned long long h[5];
        hipMemcpyAsync(h, prof, sizeof h, hipMemcpyDeviceToHost, s);
        host_sync(s);
        double tot = 0;
        for (double x : h) tot += x;
        std::fprintf(stderr, "[lsd-prof] n=%llu bits=%u packed=%d clk/tile %.0f: rank %.1f%% scan %.1f%% lookback %.1f%% stage %.1f%% write %.1f%%\n",
                     (unsigned long long)n, nbits, (int)PACKED, tot / (double)tiles,
                     100 * h[0] / tot, 100 * h[1] / tot, 100 * h[2] / tot, 100 * h[3] / tot, 100 * h[4] / tot);
    }
    return SA_OK;
}

// per-XCD queues of 8192-pair tiles (sa_lsd.h XQ): whether a sort takes
// them (unpacked passes of 10 bits do not fit their LDS with the per-queue
// counters) and the queue span
static bool lsd_xq_ok(const sa_context* c, uint64_t n, const LsdPlan& pl, bool packed) {
    const uint64_t xtiles = (n + kLsdXqTile - 1) / kLsdXqTile;
    bool xq = SA_LSD_XQ && c->cus % 8 == 0 && xtiles >= 64 && !(c->dbg & SA_DEBUG_NO_XQ);
    if (!packed)
        for (uint32_t p = 0; p < pl.P; ++p) xq = xq && pl.bits[p] <= 9;
    return xq;
}
static void lsd_xq_span(uint64_t n, uint32_t* tpq, uint64_t* qspan, QDiv* qd) {
    const uint64_t xtiles = (n + kLsdXqTile - 1) / kLsdXqTile;
    *tpq = (uint32_t)((xtiles + 7) / 8);
    *qspan = (uint64_t)*tpq * kLsdXqTile;
    qd->magic = (uint64_t)((((unsigned __int128)1 << 64) + *qspan - 1) / *qspan);
}

// Stable LSD sort of n pairs by the plan's digits, pass 0 reading `first`.
// PACKED: one item buffer ping-pong; else keys + values, the last pass
// writing its values into vals_final.  *sorted = the sorted key / item buffer.
// hist_ready (XQ): the first pass's per-queue counts are already in
// lsdx[0] (the previous round's k_perm_place counted them).
template <bool PACKED, class Src0>
static int lsd_sort(sa_context* c, const Src0& first, uint64_t n, const LsdPlan& pl, uint32_t* vals_final,
                    uint32_t* vals_other, hipStream_t s, Timer& tm, sa_stats* st, uint64_t** sorted,
                    bool hist_ready = false) {
    if (pl.P < 1 || pl.P > kMaxPasses) return set_err(SA_E_INTERNAL, "%u radix passes", pl.P);
    uint64_t* kb[2] = {c->keys[0], c->keys[1]};
    uint32_t* vb[2];
    vb[(pl.P - 1) & 1] = vals_final;
    vb[pl.P & 1] = vals_other;
    SA_HIP(hipMemsetAsync(c->lsd, 0, (2 * kMaxPasses * kLsdMaxRadix + kMaxPasses) * 4, s));
    // the first digit's totals here; every pass counts the next one's
    LsdPlan first_only = pl;
    first_only.P = 1;
    // per-XCD queues of tiles (sa_lsd.h XQ)
    if (lsd_xq_ok(c, n, pl, PACKED)) {
        uint32_t tpq;
        uint64_t qspan;
        QDiv qd;
        lsd_xq_span(n, &tpq, &qspan, &qd);
        uint32_t* const qh = c->lsdx;                                    // [pass][8][1024]
        uint32_t* const qb = qh + kMaxPasses * 8 * kLsdMaxRadix;         // [8][1024]
        uint32_t* const qt = qb + 8 * kLsdMaxRadix;                      // [pass][8 x 32]
        if (hist_ready) {   // pass 0's counts came with the previous round's re-rank
            SA_HIP(hipMemsetAsync(c->lsdx + 8 * kLsdMaxRadix, 0, (kLsdXqWords - 8 * kLsdMaxRadix) * 4, s));
        } else {
            SA_HIP(hipMemsetAsync(c->lsdx, 0, kLsdXqWords * 4, s));
            tm.begin(SA_K_HIST_FIRST);
            hipLaunchKernelGGL(k_lsd_hist<Src0>, dim3((uint32_t)std::min<uint64_t>((n + 8 * kBlock - 1) / (8 * kBlock),
                                                                                   (uint64_t)c->cus * 4)),
                               dim3(kBlock), 0, s, first, n, first_only, qh, qd);
            tm.end();
            add_bytes(st, SA_K_HIST_FIRST, 8 * n);
        }
        const uint64_t pair = PACKED ? 8 : 12;
        for (uint32_t p = 0; p < pl.P; ++p) {
            tm.begin(SA_K_SCAN);
            hipLaunchKernelGGL(k_lsd_qbase, dim3(1), dim3(1024), 0, s, (const uint32_t*)qh + p * 8 * kLsdMaxRadix,
                               1u << pl.bits[p], qb);
            tm.end();
            const bool more = p + 1 < pl.P;
            const uint32_t nsh = more ? pl.shift[p + 1] : 0u, nnb = more ? pl.bits[p + 1] : 1u;
            uint32_t* nh = more ? qh + (p + 1) * 8 * kLsdMaxRadix : nullptr;
            uint32_t* tk = qt + p * 8 * 32;
            if (p == 0) {
                tm.begin(SA_K_SCATTER_FIRST);
                SA_TRY(lsd_pass<Src0, PACKED, true>(c, first, n, pl.shift[0], pl.bits[0], qb, tk, kb[0], vb[0], s, nsh,
                                                    nnb, nh, qd, tpq));
                tm.end();
                add_bytes(st, SA_K_SCATTER_FIRST, (8 + pair) * n);
            } else {
                tm.begin(SA_K_SCATTER_KEYS);
                if constexpr (PACKED)
                    SA_TRY(lsd_pass<SrcItems, true, true>(c, SrcItems{kb[(p - 1) & 1]}, n, pl.shift[p], pl.bits[p], qb,
                                                          tk, kb[p & 1], nullptr, s, nsh, nnb, nh, qd, tpq));
                else
                    SA_TRY(lsd_pass<SrcKeys, false, true>(c, SrcKeys{kb[(p - 1) & 1], vb[(p - 1) & 1]}, n, pl.shift[p],
                                                          pl.bits[p], qb, tk, kb[p & 1], vb[p & 1], s, nsh, nnb, nh,
                                                          qd, tpq));
                tm.end();
                add_bytes(st, SA_K_SCATTER_KEYS, 2 * pair * n);
            }
        }
        SA_HIP(hipGetLastError());
        *sorted = kb[(pl.P - 1) & 1];
        return SA_OK;
    }
    tm.begin(SA_K_HIST_FIRST);
    hipLaunchKernelGGL(k_lsd_hist<Src0>, dim3((uint32_t)std::min<uint64_t>((n + 8 * kBlock - 1) / (8 * kBlock),
                                                                           (uint64_t)c->cus * 4)),
                       dim3(kBlock), 0, s, first, n, first_only, lsd_ghist(c));
    tm.end();
    add_bytes(st, SA_K_HIST_FIRST, 8 * n);
    const uint64_t pair = PACKED ? 8 : 12;
    for (uint32_t p = 0; p < pl.P; ++p) {
        uint32_t* base = lsd_base(c) + p * kLsdMaxRadix;
        tm.begin(SA_K_SCAN);
        hipLaunchKernelGGL(k_digit_base_wide, dim3(1), dim3(1024), 0, s,
                           (const uint32_t*)lsd_ghist(c) + p * kLsdMaxRadix, 1u << pl.bits[p], base);
        tm.end();
        const bool more = p + 1 < pl.P;
        const uint32_t nsh = more ? pl.shift[p + 1] : 0u, nnb = more ? pl.bits[p + 1] : 1u;
        uint32_t* nh = more ? lsd_ghist(c) + (p + 1) * kLsdMaxRadix : nullptr;
        if (p == 0) {
            tm.begin(SA_K_SCATTER_FIRST);
            SA_TRY(lsd_pass<Src0, PACKED>(c, first, n, pl.shift[0], pl.bits[0], base, lsd_tickets(c), kb[0], vb[0], s,
                                          nsh, nnb, nh));
            tm.end();
            add_bytes(st, SA_K_SCATTER_FIRST, (8 + pair) * n);
        } else {
            tm.begin(SA_K_SCATTER_KEYS);
            if constexpr (PACKED)
                SA_TRY(lsd_pass<SrcItems, true>(c, SrcItems{kb[(p - 1) & 1]}, n, pl.shift[p], pl.bits[p], base,
                                                lsd_tickets(c) + p, kb[p & 1], nullptr, s, nsh, nnb, nh));
            else
                SA_TRY(lsd_pass<SrcKeys, false>(c, SrcKeys{kb[(p - 1) & 1], vb[(p - 1) & 1]}, n, pl.shift[p],
                                                pl.bits[p], base, lsd_tickets(c) + p, kb[p & 1], vb[p & 1], s, nsh,
                                                nnb, nh));
            tm.end();
            add_bytes(st, SA_K_SCATTER_KEYS, 2 * pair * n);
        }
    }
    SA_HIP(hipGetLastError());
    *sorted = kb[(pl.P - 1) & 1];
    return SA_OK;
}

// round 1's first-digit counts taken by the init kernel (A/B switch)
#ifndef SA_INIT_HIST
#define SA_INIT_HIST 1
#endif
static int build_reference(sa_context* c, const uint8_t* d_text, uint64_t n, uint32_t* d_sa, hipStream_t s,
                           sa_stats* st, Timer& tm) {
    int rc = SA_OK;
    const Chunking ch = plan_chunks(n);
    // first ranks: dense codes 1..sigma of the bytes present (the order of
    // manber_myers.c:90's text[i] + 1, so D_j and the round count are the
    // reference's; the first key spans 2 bit_width(sigma) bits, not 18)
    uint32_t* h_alpha = c->host_words + 64;
    uint16_t* h_code = reinterpret_cast<uint16_t*>(c->host_words + 320);
    SA_HIP(hipMemsetAsync(c->alpha, 0, 8 * 4, s));
    tm.begin(SA_K_ALPHABET);
    {
        const uint32_t grid = (uint32_t)std::min<uint64_t>((n + kBlock * 16 - 1) / (kBlock * 16), SA_ALPHA_GRID);
        hipLaunchKernelGGL(k_alphabet, dim3(grid), dim3(kBlock), 0, s, d_text, n, c->alpha);
    }
    tm.end();
    add_bytes(st, SA_K_ALPHABET, n);
    SA_HIP(hipMemcpyAsync(h_alpha, c->alpha, 8 * 4, hipMemcpyDeviceToHost, s));
    SA_HIP(host_sync(s));
    uint32_t sigma = 0;
    for (int b = 0; b < 256; ++b) h_code[b] = ((h_alpha[b >> 5] >> (b & 31)) & 1u) ? (uint16_t)(++sigma) : 0;
    SA_HIP(hipMemcpyAsync(c->code, h_code, 256 * 2, hipMemcpyHostToDevice, s));
    uint64_t D = sigma;   // ranks 1..sigma (manber_myers.c:94 sizes its bins for 256)
    const uint64_t perm_min = perm_min_n(c);
    const uint32_t ib = std::max<uint32_t>(1, bit_width(n - 1));   // index bits of a packed item
    bool used_perm = false;
    bool hist_ready = false;   // this round's first-digit counts came with the previous re-rank (or the init)
    tm.begin(SA_K_INIT);
    {
        // round 1's first-digit counts per XCD queue with the ranks (k_init_rank_hist)
        const uint32_t w1 = bit_width(D);
        const bool packed1 = c->radix == 0 && 2 * w1 + ib <= 64;
        const LsdPlan pl1 = lsd_plan(2 * w1, packed1 ? ib : 0, lsd_max_bits(c));
        if (SA_INIT_HIST && c->radix == 0 && lsd_xq_ok(c, n, pl1, packed1)) {
            uint32_t tpq;
            uint64_t qspan;
            QDiv qd;
            lsd_xq_span(n, &tpq, &qspan, &qd);
            SA_HIP(hipMemsetAsync(c->lsdx, 0, 8 * kLsdMaxRadix * 4, s));
            const uint64_t grid = std::min<uint64_t>((n + kBlock * 16 - 1) / (kBlock * 16), 4ull * (uint64_t)c->cus);
            hipLaunchKernelGGL(k_init_rank_hist, dim3((uint32_t)grid), dim3(kBlock), 0, s, d_text, n,
                               (const uint16_t*)c->code, c->rank, w1, pl1.shift[0] - (packed1 ? ib : 0u),
                               (1u << pl1.bits[0]) - 1u, qd, c->lsdx);
            hist_ready = true;
        } else {
            const uint64_t grid = std::min<uint64_t>((n + kBlock * 4 - 1) / (kBlock * 4), 4096);
            hipLaunchKernelGGL(k_init_rank_dense, dim3((uint32_t)grid), dim3(kBlock), 0, s, d_text, n,
                               (const uint16_t*)c->code, c->rank);
        }
    }
    tm.end();
    SA_HIP(hipGetLastError());
    add_bytes(st, SA_K_INIT, 5 * n);
    if (st) st->sigma = (int32_t)sigma;

    tm.round_mark();
    for (uint64_t h = 1;; h *= 2) {
        const uint32_t w = bit_width(D);          // ranks are 0..D
        // (key << ib | index) items while they fit 64 bits (onesweep only)
        const bool packed = c->radix == 0 && 2 * w + ib <= 64;
        SA_TRACE("reference round h=%llu D=%llu w=%u%s", (unsigned long long)h, (unsigned long long)D, w,
                 packed ? " packed" : "");
        SrcRank src{c->rank, n, h, w};
        uint64_t* sorted;
        uint32_t P;
        if (c->radix == 0) {
            const LsdPlan pl = lsd_plan(2 * w, packed ? ib : 0, lsd_max_bits(c));
            P = pl.P;
            rc = packed ? lsd_sort<true>(c, SrcRankPk{c->rank, n, h, w, ib}, n, pl, d_sa, c->vals_alt, s, tm, st,
                                         &sorted, hist_ready)
                        : lsd_sort<false>(c, src, n, pl, d_sa, c->vals_alt, s, tm, st, &sorted, hist_ready);
        } else {
            rc = radix_sort(c, src, 4 * n, ch, 2 * w, d_sa, c->vals_alt, c->keys[0], c->keys[1], s, tm, st, &sorted,
                            &P);
        }
        if (rc) return rc;
        // the permutation's first level counts heads per tile of its own
        const bool use_perm = packed || n >= perm_min;
        const uint32_t ptiles = (uint32_t)((n + kPermTile - 1) / kPermTile);
        tm.begin(SA_K_HEADS);
        if (use_perm)
            hipLaunchKernelGGL((k_tile_heads<kPermBlock, kPermItems>), dim3(ptiles), dim3(kPermBlock), 0, s,
                               (const uint64_t*)sorted, n, packed ? ib : 0u, perm_tile_off(c));
        else
            hipLaunchKernelGGL(k_heads, dim3(ch.chunks), dim3(kBlock), 0, s, sorted, ch, c->counts, 0u);
        tm.end();
        tm.begin(SA_K_HEADS_SCAN);
        if (use_perm)
            hipLaunchKernelGGL(k_scan_heads, dim3(1), dim3(kBlock), 0, s, perm_tile_off(c), ptiles, c->words);
        else
            hipLaunchKernelGGL(k_scan_heads, dim3(1), dim3(kBlock), 0, s, c->counts, ch.chunks, c->words);
        tm.end();
        SA_HIP(hipGetLastError());
        add_bytes(st, SA_K_HEADS, 8 * n);
        add_bytes(st, SA_K_HEADS_SCAN, 8ull * ch.chunks);
        // (with the permutation re-rank's error word: the previous round's
        // placement is checked before this round's ranks are used)
        SA_HIP(hipMemcpyAsync(c->host_words, c->words, 4 * (kPermErrWord + 1), hipMemcpyDeviceToHost, s));
        SA_HIP(host_sync(s));
        if (c->host_words[4]) return set_err(SA_E_INTERNAL, "radix look-back did not complete");
        if (used_perm && c->host_words[kPermErrWord])
            return set_err(SA_E_INTERNAL, "re-rank permutation lost a suffix (flags %u)", c->host_words[kPermErrWord]);
        const uint64_t Dn = c->host_words[0];
        const bool done = (Dn == n);                  // manber_myers.c:113
        if (done && packed) {
            tm.begin(SA_K_RERANK);
            hipLaunchKernelGGL(k_items_to_sa, dim3((uint32_t)std::min<uint64_t>((n + kBlock - 1) / kBlock, 8192)),
                               dim3(kBlock), 0, s, (const uint64_t*)sorted, n, ib, d_sa);
            tm.end();
            SA_HIP(hipGetLastError());
            add_bytes(st, SA_K_RERANK, 12 * n);
        }
        hist_ready = false;
        if (!done) {
            if (use_perm) {
                used_perm = true;
                // the next round's first digit lies in rank[i + 2h] alone (its
                // width <= w'): the re-rank counts it per queue of that round's
                // LSD passes while it writes rank[] (no histogram read then)
                NextHist nh;
                if (c->radix == 0) {
                    const uint32_t w2 = bit_width(Dn);
                    const bool packed2 = 2 * w2 + ib <= 64;
                    const LsdPlan pl2 = lsd_plan(2 * w2, packed2 ? ib : 0, lsd_max_bits(c));
                    if (pl2.bits[0] <= w2 && lsd_xq_ok(c, n, pl2, packed2)) {
                        uint32_t tpq;
                        lsd_xq_span(n, &tpq, &nh.qspan, &nh.qd);
                        nh.out = c->lsdx;
                        nh.mask = (1u << pl2.bits[0]) - 1u;
                        nh.h = 2 * h;
                        hist_ready = true;
                    }
                }
                rc = rerank_permute(c, sorted, d_sa, ch, s, tm, st, packed ? ib : 0u, nh);
                if (rc) return rc;
            } else {
                tm.begin(SA_K_RERANK);
                hipLaunchKernelGGL(k_rerank, dim3(ch.chunks), dim3(kBlock), 0, s, sorted, (const uint32_t*)d_sa, ch,
                                   (const uint32_t*)c->counts, c->rank);
                tm.end();
                SA_HIP(hipGetLastError());
                add_bytes(st, SA_K_RERANK, 16 * n);
            }
        }
        tm.round_mark();
        record_round(st, 0.f, Dn, P, n, 2 * h);   // (its time: Timer::round_times)
        if (Dn > n || Dn == 0)
            return set_err(SA_E_INTERNAL, "distinct count %llu out of range", (unsigned long long)Dn);
        if (done) break;
        if (h > n) return set_err(SA_E_INTERNAL, "doubling did not converge (h=%llu)", (unsigned long long)h);
        D = Dn;
    }
    if (used_perm) {
        SA_HIP(hipMemcpyAsync(c->host_words + kPermErrWord, c->words + kPermErrWord, 4, hipMemcpyDeviceToHost, s));
        SA_HIP(host_sync(s));
        if (c->host_words[kPermErrWord])
            return set_err(SA_E_INTERNAL, "re-rank permutation lost a suffix (flags %u)", c->host_words[kPermErrWord]);
    }
    return SA_OK;
}

// ---------------------------------------------------------------------------
// packed schedule
// ---------------------------------------------------------------------------
// K for base B: largest K with B^K - 1 < 2^64
static uint32_t max_chars(uint64_t base) {
    uint32_t K = 0;
    uint64_t prod = 1;
    while (prod <= UINT64_MAX / base) {
        prod *= base;
        ++K;
    }
    return K;
}

static uint32_t key_bits(uint64_t base, uint32_t K) {   // bit width of B^K - 1
    unsigned __int128 p = 1;
    for (uint32_t t = 0; t < K; ++t) p *= base;
    p -= 1;
    uint32_t w = 0;
    while (p) { ++w; p >>= 1; }
    return w;
}

// the fewest symbols K with sigma^K >= 512 n: a random text of this
// alphabet then leaves few suffixes unsorted by round 1
static uint32_t min_chars(uint32_t sigma, uint64_t n) {
    const uint32_t kmax = max_chars((uint64_t)sigma + 1);
    uint32_t kmin = 1;
    unsigned __int128 p = sigma, target = (unsigned __int128)n * 512u;
    while (p < target && kmin < kmax) {
        p *= sigma;
        ++kmin;
    }
    return kmin;
}

// auto K: min_chars, rounded up to fill the radix passes (the LSD round 1).
static uint32_t choose_chars(uint32_t sigma, uint64_t n, int32_t req) {
    const uint64_t base = (uint64_t)sigma + 1;
    const uint32_t kmax = max_chars(base);
    if (req > 0) return std::min<uint32_t>((uint32_t)req, kmax);
    if (sigma <= 1) return kmax;
    const uint32_t kmin = min_chars(sigma, n);
    const uint32_t P = (key_bits(base, kmin) + 7) / 8;
    uint32_t K = kmin;
    while (K + 1 <= kmax && key_bits(base, K + 1) <= 8 * P) ++K;
    return K;
}

// unsorted-set rounds try the per-group register sort when the average
// group holds at most kUsAvg suffixes; its oversize flag lives in words[12]
constexpr uint64_t kUsAvg = 4;
// per-group register sort over keys materialised one lane per suffix first
#ifndef SA_US_TWO_PHASE
#define SA_US_TWO_PHASE 1
#endif
constexpr int kUsFlagWord = 12;

template <class Pos>
static int segments(sa_context* c, const uint64_t* keys, const uint32_t* idx, const Chunking& ch, Pos pos,
                    bool sparse_ok, bool* sparse_out,
                    uint32_t* sa, int uo, hipStream_t s, Timer& tm, sa_stats* st, uint64_t* D, uint64_t* m,
                    uint64_t* G, uint32_t* rank_arr = nullptr, uint64_t rank_off = 0, RankMap rm = RankMap{},
                    uint64_t set_off = 0, uint32_t g_off = 0, uint32_t* gsn = nullptr) {
    // rank_arr / rank_off / rm: the range-partitioned build's compact rank map
    // and its SA offset (sa_dist.h); the context's rank array, 0 and the
    // identity map on one GPU.  set_off / g_off: the next unsorted set's
    // first slot and group id (the tied-block round's rest, sa_pivot.h)
    if (!rank_arr) rank_arr = c->rank;
    uint32_t* c_h = c->counts;
    uint32_t* c_u = c->counts + kMaxChunks;
    uint32_t* c_uh = c->counts + 2 * kMaxChunks;
    uint32_t* c_l = c->counts + 3 * kMaxChunks;
    tm.begin(SA_K_SEG_COUNT);
    hipLaunchKernelGGL(k_seg_count, dim3(ch.chunks), dim3(kBlock), 0, s, keys, ch, c_h, c_u, c_uh, c_l);
    tm.end();
    tm.begin(SA_K_SEG_SCAN);
    hipLaunchKernelGGL(k_seg_scan, dim3(1), dim3(kBlock), 0, s, c_h, c_u, c_uh, c_l, ch.chunks, c->words);
    tm.end();
    SA_HIP(hipGetLastError());
    SA_HIP(hipMemcpyAsync(c->host_words, c->words, 20, hipMemcpyDeviceToHost, s));
    SA_HIP(host_sync(s));
    if (c->host_words[4]) return set_err(SA_E_INTERNAL, "radix look-back did not complete");
    *D = c->host_words[0];
    *m = c->host_words[1];
    *G = c->host_words[2];
    // first round with few unsorted suffixes: keep ranks only for those
    const bool sparse = sparse_ok && *m <= ch.n / kSparseDiv;
    uint32_t* member = nullptr;
    if (sparse) {
        SA_HIP(hipMemsetAsync(c->member, 0, (ch.n + 31) / 32 * 4, s));
        member = c->member;
    }
    if (sparse_out) *sparse_out = sparse;
    tm.begin(SA_K_SEG_WRITE);
    hipLaunchKernelGGL(k_seg_write<Pos>, dim3(ch.chunks), dim3(kBlock), 0, s, keys, idx, ch, pos,
                       (const uint32_t*)c_u, (const uint32_t*)c_uh, (const uint32_t*)c_l, rank_arr, sa,
                       c->u_pos[uo] + set_off, c->u_idx[uo] + set_off, c->u_g[uo] + set_off, member, sparse ? 0 : 1,
                       (uint32_t)rank_off, rm, g_off, gsn ? gsn + g_off : nullptr, (uint32_t)set_off);
    tm.end();
    SA_HIP(hipGetLastError());
    add_bytes(st, SA_K_SEG_COUNT, 8 * ch.n);
    add_bytes(st, SA_K_SEG_SCAN, 32ull * ch.chunks);
    add_bytes(st, SA_K_SEG_WRITE, ch.n * (8 + (sparse ? 0 : 8)) + (sa ? 8 * ch.n : 0) + *m * 16);
    return SA_OK;
}

// Unsorted-set round by a three-way pivot split (sa_pivot.h): dense ranks,
// large groups on average.  Returns SA_OK with *sorted = nullptr when the
// tied blocks turn out small (the caller then sorts the whole set).
static bool pivot_ok(const sa_context* c, uint64_t m, uint64_t G, uint32_t wr, bool sparse) {
    return !(c->dbg & SA_DEBUG_NO_PIVOT) && c->radix == 0 && !sparse && m >= (1u << 16) && G >= 1 && G <= m / 4 && bit_width(2 * G + 1) + wr <= 64;
}

// keys + class counts of a pivot round in one pass when the set came with its
// group starts (sa_pivot.h MODE 1; A/B switch)
#ifndef SA_PIVOT_MERGED
#define SA_PIVOT_MERGED 1
#endif
// tied-block rounds (sa_pivot.h) scan the groups in one workgroup
constexpr uint64_t kPivotTiedMaxG = 1u << 18;

static int pivot_round(sa_context* c, int ui, int uo, uint64_t n, uint64_t m, uint64_t G, uint64_t h, uint32_t wr,
                       uint64_t* ukb0, uint64_t* ukb1, uint64_t* kbA, const Chunking& cu, uint32_t* d_sa,
                       hipStream_t s, Timer& tm, sa_stats* st, uint64_t** sorted, uint32_t* P, bool* segs_done,
                       uint64_t* Du, uint64_t* m2, uint64_t* G2, bool have_gs, bool* gs_written) {
    // have_gs: the set's group starts are in u_gs[ui] (written with it by the
    // previous round); *gs_written: this round wrote the next set's to u_gs[uo]
    *sorted = nullptr;
    *segs_done = false;
    *gs_written = false;
    // tied-block round: its scratch is ukb0 (free: the tied members skip the
    // sorted output) -- gs, pr, toff, tid, then the rest's values (3 x
    // m' <= 3 m / 2 words)
    const uint64_t scap = 2 * align_up(c->cap, 64);
    const uint64_t sbase = align_up(4 * G + 3, 64);
    const uint64_t ra_max = align_up(m / 2, 64);
    // tied blocks write the next set's group starts: u_gs is allocated here,
    // and a workspace too tight for it takes the split path (k_pivot_pass<2>,
    // no extra memory) instead of failing the build
    const bool tied = !(c->dbg & SA_DEBUG_NO_TIED) && G <= kPivotTiedMaxG && sbase + 3 * ra_max <= scap &&
                      gs_available(c, n);
    uint32_t* const scr = reinterpret_cast<uint32_t*>(ukb0);
    const bool merged = SA_PIVOT_MERGED && tied && have_gs;
    uint32_t* const gs = merged ? c->u_gs[ui] : tied ? scr : c->u_pos[uo];   // G (+ 1) group starts
    uint32_t* const pr = (tied ? scr : gs) + G + 1;                          // G pivot ranks
    uint32_t* const gP = c->vals_alt;                 // 3 (G + 1): members of each class before each group
    uint32_t* const cc = c->hist;                     // 3 x chunks class counts, scanned in place
    const uint32_t Gu = (uint32_t)G;
    if (merged) {
        // the group starts came with the set: keys built and classes counted
        // in one pass (MODE 1: k_pivot_keys + MODE 0)
        tm.begin(SA_K_PIVOT_COUNT);
        PivotKeySrc ks;
        ks.rank = c->rank;
        ks.n = n;
        ks.h = h;
        ks.keys_out = ukb1;
        ks.pr_out = pr;
        hipLaunchKernelGGL(k_pivot_pass<1>, dim3(cu.chunks), dim3(kBlock), 0, s, (const uint64_t*)nullptr,
                           (const uint32_t*)c->u_idx[ui], (const uint32_t*)c->u_g[ui], cu, (const uint32_t*)gs,
                           (const uint32_t*)pr, Gu, wr, cc, gP, nullptr, nullptr, nullptr, nullptr, TiedOut{}, ks);
        hipLaunchKernelGGL(k_scan_rows, dim3(3), dim3(kBlock), 0, s, cc, cu.chunks, c->totals);
        tm.end();
        SA_HIP(hipGetLastError());
        add_bytes(st, SA_K_PIVOT_COUNT, 20 * m);
    } else {
        tm.begin(SA_K_PIVOT_KEYS);
        hipLaunchKernelGGL(k_pivot_keys,
                           dim3((uint32_t)std::min<uint64_t>((m + kBlock * kPkItems - 1) / (kBlock * kPkItems), 8192)),
                           dim3(kBlock), 0, s, (const uint32_t*)c->u_idx[ui], (const uint32_t*)c->u_g[ui], m,
                           (const uint32_t*)c->rank, n, h, wr, Gu, ukb1, gs, pr);
        tm.end();
        add_bytes(st, SA_K_PIVOT_KEYS, 20 * m);
        tm.begin(SA_K_PIVOT_COUNT);
        hipLaunchKernelGGL(k_pivot_pass<0>, dim3(cu.chunks), dim3(kBlock), 0, s, (const uint64_t*)ukb1,
                           (const uint32_t*)c->u_idx[ui], (const uint32_t*)c->u_g[ui], cu, (const uint32_t*)gs,
                           (const uint32_t*)pr, Gu, wr, cc, gP, nullptr, nullptr, nullptr, nullptr, TiedOut{});
        hipLaunchKernelGGL(k_scan_rows, dim3(3), dim3(kBlock), 0, s, cc, cu.chunks, c->totals);
        tm.end();
        SA_HIP(hipGetLastError());
        add_bytes(st, SA_K_PIVOT_COUNT, 8 * m);
    }
    SA_HIP(hipMemcpyAsync(c->host_words + 16, c->totals, 12, hipMemcpyDeviceToHost, s));
    SA_HIP(host_sync(s));
    const uint64_t t0 = c->host_words[16], t1 = c->host_words[17], t2 = c->host_words[18];
    if (t0 + t1 + t2 != m) return set_err(SA_E_INTERNAL, "pivot classes %llu + %llu + %llu != %llu",
                                          (unsigned long long)t0, (unsigned long long)t1, (unsigned long long)t2,
                                          (unsigned long long)m);
    SA_TRACE("  round h=%llu: pivot split, tied %llu of %llu%s", (unsigned long long)h, (unsigned long long)t1,
             (unsigned long long)m, tied ? " (tied blocks to the next set)" : "");
    if (t1 * 2 < m) return SA_OK;   // mostly distinct keys: the full sort is cheaper
    tm.begin(SA_K_PIVOT_WRITE);
    hipLaunchKernelGGL(k_pivot_gp, dim3((uint32_t)std::min<uint64_t>((G + kBlock) / kBlock, 8192)), dim3(kBlock), 0, s,
                       (const uint32_t*)gs, Gu, (const uint32_t*)cc, cu, (const uint32_t*)c->totals, gP);
    const uint64_t mr = t0 + t2;
    const uint64_t ra = align_up(mr, 64);
    uint32_t* const ridx = tied ? scr + sbase : c->u_idx[uo];
    uint64_t T = 0, Gt = 0, Dt = 0;
    if (tied) {
        // the next set's group starts go with it (the next pivot round's MODE 1;
        // u_gs allocated by gs_available above)
        uint32_t* const toff = scr + 2 * G + 1;
        uint32_t* const tid = toff + G + 1;
        hipLaunchKernelGGL(k_pivot_tied_scan, dim3(1), dim3(kBlock), 0, s, (const uint32_t*)gP, Gu, toff, tid,
                           c->totals + 4);
        const TiedOut to{c->u_pos[ui], toff, tid, c->rank, d_sa, c->u_pos[uo], c->u_idx[uo], c->u_g[uo], c->u_gs[uo]};
        hipLaunchKernelGGL(k_pivot_pass<3>, dim3(cu.chunks), dim3(kBlock), 0, s, (const uint64_t*)ukb1,
                           (const uint32_t*)c->u_idx[ui], (const uint32_t*)c->u_g[ui], cu, (const uint32_t*)gs,
                           (const uint32_t*)pr, Gu, wr, cc, gP, nullptr, nullptr, kbA, ridx, to);
    } else {
        hipLaunchKernelGGL(k_pivot_pass<2>, dim3(cu.chunks), dim3(kBlock), 0, s, (const uint64_t*)ukb1,
                           (const uint32_t*)c->u_idx[ui], (const uint32_t*)c->u_g[ui], cu, (const uint32_t*)gs,
                           (const uint32_t*)pr, Gu, wr, cc, gP, ukb0, c->vals_u, kbA, ridx, TiedOut{});
    }
    tm.end();
    SA_HIP(hipGetLastError());
    add_bytes(st, SA_K_PIVOT_WRITE, tied ? 12 * m + 16 * t1 + 12 * mr : 12 * m + 12 * m);
    if (tied) {
        SA_HIP(hipMemcpyAsync(c->host_words + 20, c->totals + 4, 12, hipMemcpyDeviceToHost, s));
        SA_HIP(host_sync(s));
        T = c->host_words[20];
        Gt = c->host_words[21];
        Dt = c->host_words[22];
        if (T > t1 || Gt > G || Dt > G)
            return set_err(SA_E_INTERNAL, "tied blocks %llu / %llu / %llu out of range", (unsigned long long)T,
                           (unsigned long long)Gt, (unsigned long long)Dt);
    }
    uint32_t Pr = 0;
    uint64_t Dr = 0, mrr = 0, Gr = 0;
    if (mr > 0) {
        // the rest sorted by (2 g + [> pivot], rank): values in u_idx / u_g
        // of the next set (free until segments()) or the tied round's
        // scratch, keys through kbA and ukb1
        const uint32_t bits = bit_width(2 * G - 1) + wr;
        const uint32_t Pn = (bits + 7) / 8;
        uint32_t* const va = tied ? ridx + ra : c->u_g[uo];
        uint32_t* const vb = tied ? ridx + 2 * ra : c->u_idx[uo];
        uint32_t* vfinal = (Pn & 1u) ? va : vb;
        uint32_t* vother = (Pn & 1u) ? vb : va;
        uint64_t* rs = nullptr;
        int rc = radix_sort(c, SrcKeys{kbA, ridx}, 12 * mr, plan_chunks(mr), bits, vfinal, vother, ukb1, kbA, s, tm,
                            st, &rs, &Pr, false, true);
        if (rc) return rc;
        tm.begin(SA_K_SORT_U);
        const dim3 pg((uint32_t)std::min<uint64_t>((mr + kBlock - 1) / kBlock, 8192));
        if (tied)
            hipLaunchKernelGGL(k_pivot_place<true>, pg, dim3(kBlock), 0, s, (const uint64_t*)rs,
                               (const uint32_t*)vfinal, mr, (const uint32_t*)gs, (const uint32_t*)gP, Gu, wr, nullptr,
                               nullptr, m, (const uint32_t*)c->u_pos[ui], c->vals_u);
        else
            hipLaunchKernelGGL(k_pivot_place<false>, pg, dim3(kBlock), 0, s, (const uint64_t*)rs,
                               (const uint32_t*)vfinal, mr, (const uint32_t*)gs, (const uint32_t*)gP, Gu, wr, ukb0,
                               c->vals_u, m, nullptr, nullptr);
        tm.end();
        SA_HIP(hipGetLastError());
        add_bytes(st, SA_K_SORT_U, tied ? 20 * mr : 24 * mr);
        if (tied) {
            // the rest's segments, appended to the next set after the tied blocks
            rc = segments(c, rs, vfinal, plan_chunks(mr), PosArray{c->vals_u}, false, nullptr, d_sa, uo, s, tm, st,
                          &Dr, &mrr, &Gr, nullptr, 0, RankMap{}, T, (uint32_t)Gt, c->u_gs[uo]);
            if (rc) return rc;
        }
    }
    *P = 1 + Pr;
    if (tied) {
        *gs_written = true;
        *segs_done = true;
        *Du = Dr + Dt;
        *m2 = mrr + T;
        *G2 = Gr + Gt;
    }
    *sorted = ukb0;
    return SA_OK;
}

// Round 1 by the pivot split (sa_pivot.h, R1): when the LSD round 1 would
// run and at least half of all suffixes share the key of suffix 0 (a text of
// one repeated symbol, configs[4]: all but the last K), those form one tied
// block -- ranks and the next unsorted set written directly -- and only the
// rest is radix sorted (then segments() over it, SA positions around the
// block's gap).  *done = false (nothing written but the class counts) when
// fewer share it: the caller runs the LSD sort.
static int pivot_round1(sa_context* c, uint64_t n, uint32_t bits1, uint32_t* d_sa, hipStream_t s, Timer& tm,
                        sa_stats* st, bool* done, uint64_t* D, uint64_t* m, uint64_t* G, uint32_t* P) {
    *done = false;   // (done: the set's group starts are in u_gs[0] too)
    const Chunking ch = plan_chunks(n);
    const uint64_t* keys = c->keys[1];
    uint32_t* const gs = c->u_pos[1];   // {0, n}: one group
    uint32_t* const toff = gs + 2;
    uint32_t* const tid = gs + 4;
    uint32_t* const gP = c->vals_alt;   // 3 x 2
    uint32_t* const cc = c->hist;       // 3 x chunks class counts
    c->host_words[24] = 0;
    c->host_words[25] = (uint32_t)n;
    SA_HIP(hipMemcpyAsync(gs, c->host_words + 24, 8, hipMemcpyHostToDevice, s));
    tm.begin(SA_K_PIVOT_COUNT);
    hipLaunchKernelGGL((k_pivot_pass<0, true>), dim3(ch.chunks), dim3(kBlock), 0, s, keys, nullptr, nullptr, ch,
                       (const uint32_t*)gs, nullptr, 1u, 0u, cc, gP, nullptr, nullptr, nullptr, nullptr, TiedOut{});
    hipLaunchKernelGGL(k_scan_rows, dim3(3), dim3(kBlock), 0, s, cc, ch.chunks, c->totals);
    tm.end();
    SA_HIP(hipGetLastError());
    add_bytes(st, SA_K_PIVOT_COUNT, 8 * n);
    SA_HIP(hipMemcpyAsync(c->host_words + 16, c->totals, 12, hipMemcpyDeviceToHost, s));
    SA_HIP(host_sync(s));
    const uint64_t t0 = c->host_words[16], t1 = c->host_words[17], t2 = c->host_words[18];
    if (t0 + t1 + t2 != n) return set_err(SA_E_INTERNAL, "round-1 pivot classes %llu + %llu + %llu != %llu",
                                          (unsigned long long)t0, (unsigned long long)t1, (unsigned long long)t2,
                                          (unsigned long long)n);
    SA_TRACE("  round 1: pivot split, tied %llu of %llu", (unsigned long long)t1, (unsigned long long)n);
    if (t1 * 2 < n) return SA_OK;
    const uint64_t mr = t0 + t2;
    // the rest: keys -> keys[0], values ping-pong in u_idx[1] / u_g[1] (the
    // next set goes to u_*[0]), key buffers keys_u / keys[0]
    uint64_t* const rk = c->keys[0];
    uint32_t* const ridx = c->u_idx[1];
    // the set's group starts, for round 2's MODE 1; without room for them
    // round 1 keeps the LSD sort (*done = false: nothing written yet)
    if (!gs_available(c, n)) return SA_OK;
    tm.begin(SA_K_PIVOT_WRITE);
    hipLaunchKernelGGL(k_pivot_gp, dim3(1), dim3(kBlock), 0, s, (const uint32_t*)gs, 1u, (const uint32_t*)cc, ch,
                       (const uint32_t*)c->totals, gP);
    hipLaunchKernelGGL(k_pivot_tied_scan, dim3(1), dim3(kBlock), 0, s, (const uint32_t*)gP, 1u, toff, tid,
                       c->totals + 4);
    const TiedOut to{nullptr, toff, tid, c->rank, d_sa, c->u_pos[0], c->u_idx[0], c->u_g[0], c->u_gs[0]};
    hipLaunchKernelGGL((k_pivot_pass<3, true>), dim3(ch.chunks), dim3(kBlock), 0, s, keys, nullptr, nullptr, ch,
                       (const uint32_t*)gs, nullptr, 1u, 0u, cc, gP, nullptr, nullptr, rk, ridx, to);
    tm.end();
    SA_HIP(hipGetLastError());
    add_bytes(st, SA_K_PIVOT_WRITE, 8 * n + 16 * t1 + 12 * mr);
    SA_HIP(hipMemcpyAsync(c->host_words + 20, c->totals + 4, 12, hipMemcpyDeviceToHost, s));
    SA_HIP(host_sync(s));
    const uint64_t T = c->host_words[20], Gt = c->host_words[21], Dt = c->host_words[22];
    if (T > t1 || Gt > 1 || Dt > 1)
        return set_err(SA_E_INTERNAL, "round-1 tied block %llu / %llu / %llu out of range", (unsigned long long)T,
                       (unsigned long long)Gt, (unsigned long long)Dt);
    uint32_t Pr = 0;
    uint64_t Dr = 0, mrr = 0, Gr = 0;
    if (mr > 0) {
        const uint32_t Pn = (bits1 + 7) / 8;
        uint32_t* const vfinal = (Pn & 1u) ? c->u_g[1] : ridx;
        uint32_t* const vother = (Pn & 1u) ? ridx : c->u_g[1];
        uint64_t* rs = nullptr;
        int rc = radix_sort(c, SrcKeys{rk, ridx}, 12 * mr, plan_chunks(mr), bits1, vfinal, vother, c->keys_u, rk, s,
                            tm, st, &rs, &Pr);
        if (rc) return rc;
        rc = segments(c, rs, vfinal, plan_chunks(mr), PosGap{t0, t1}, false, nullptr, d_sa, 0, s, tm, st, &Dr, &mrr,
                      &Gr, nullptr, 0, RankMap{}, T, (uint32_t)Gt, c->u_gs[0]);
        if (rc) return rc;
    }
    *done = true;
    *D = Dr + Dt;
    *m = mrr + T;
    *G = Gr + Gt;
    *P = 2 + Pr;
    return SA_OK;
}

static int build_packed(sa_context* c, const uint8_t* d_text, uint64_t n, uint32_t* d_sa, hipStream_t s,
                        const sa_opts* opts, sa_stats* st, Timer& tm) {
    int rc = SA_OK;
    rc = ensure_u_capacity(c, n);
    if (rc) return rc;
    tm.round_mark();
    // alphabet -> dense codes (host reads the 256-bit presence mask)
    uint32_t* h_alpha = c->host_words + 64;
    uint16_t* h_code = reinterpret_cast<uint16_t*>(c->host_words + 320);
    SA_HIP(hipMemsetAsync(c->alpha, 0, 8 * 4, s));
    tm.begin(SA_K_ALPHABET);
    {
        const uint32_t grid = (uint32_t)std::min<uint64_t>((n + kBlock * 16 - 1) / (kBlock * 16), SA_ALPHA_GRID);
        hipLaunchKernelGGL(k_alphabet, dim3(grid), dim3(kBlock), 0, s, d_text, n, c->alpha);
    }
    tm.end();
    SA_HIP(hipGetLastError());
    add_bytes(st, SA_K_ALPHABET, n);
    SA_HIP(hipMemcpyAsync(h_alpha, c->alpha, 8 * 4, hipMemcpyDeviceToHost, s));
    // the text's last bytes: the compact key layout's check (short_suffix_ties)
    const uint32_t tail_n = (uint32_t)std::min<uint64_t>(n, (uint64_t)kMaxK);
    uint8_t* h_tail = reinterpret_cast<uint8_t*>(c->host_words + 2048);
    SA_HIP(hipMemcpyAsync(h_tail, d_text + (n - tail_n), tail_n, hipMemcpyDeviceToHost, s));
    SA_HIP(host_sync(s));
    uint32_t sigma = 0;
    for (int b = 0; b < 256; ++b) h_code[b] = ((h_alpha[b >> 5] >> (b & 31)) & 1u) ? (uint16_t)(++sigma) : 0;
    SA_HIP(hipMemcpyAsync(c->code, h_code, 256 * 2, hipMemcpyHostToDevice, s));
    c->dna = sigma == 4 && h_code['A'] && h_code['C'] && h_code['G'] && h_code['T'];
    uint32_t K = choose_chars(sigma, n, opts ? opts->init_chars : 0);
    const uint64_t base = (uint64_t)sigma + 1;
    const Chunking ch = plan_chunks(n);
    uint64_t* keys1 = nullptr;
    uint32_t ksh1 = 0;   // bucketed round 1: keys1 holds every 2^ksh1-th sorted key1
    c->samples_pending = false;
    uint32_t P = 0;

    // round 1: sort every suffix by its first K symbols -- bucketed (two
    // global passes + per-window LDS sort) when the text allows it, else the
    // LSD sort of the packed key
    BucketPlan bp;
    const int r1 = opts ? opts->round1 : SA_ROUND1_AUTO;
    // the bucketed round sorts by min_chars symbols (an explicit K as given):
    // rounding K up to fill radix passes only serves the LSD round, and a
    // shorter key1 keeps its low bits narrow enough for the fixed-span local
    // sort and the per-XCD second pass (1 GiB alnum: K 8 -> 7, 16.05 -> 13.59
    // ms, profiles/r06_h_bench_alnum_k*.log; DNA, ascii127, byte256: the same K)
    const uint32_t Kb = (opts && opts->init_chars > 0) || sigma <= 1 ? K : min_chars(sigma, n);
    bool bucketed = plan_bucketed(sigma, n, Kb, r1, c->radix, &bp, 1, (c->dbg & SA_DEBUG_NO_CMP) ? 0 : 1);
    if (bucketed && bp.bs.cmp && short_suffix_ties(h_tail, n, tail_n, h_code, sigma, bp.bs.s, bp.bs.R))
        bucketed = plan_bucketed(sigma, n, Kb, r1, c->radix, &bp, 1, 0);
    // a non-power-of-two alphabet one bit short of packed first-pass items
    // (1 GiB alnum / ascii127: 65 bits) takes the E-only layout when the
    // text's last K suffixes pad apart (BucketSpec, sa_kernels.h)
    const bool force_eonly = (c->dbg & SA_DEBUG_EONLY) != 0;
    if (bucketed && bp.bs.cmp == 1 && ((sigma & (sigma - 1)) != 0 || force_eonly) && !(c->dbg & SA_DEBUG_NO_EONLY)) {
        const uint32_t hb = bp.bs.bb - kLoBits;
        BucketPlan b2;
        if ((force_eonly || !plan_pk8(bp, hb, c->dbg, true)) && plan_bucketed(sigma, n, Kb, r1, c->radix, &b2, 1, 2) &&
            (force_eonly || plan_pk8(b2, hb, c->dbg, true)) &&
            !short_suffix_ties(h_tail, n, tail_n, h_code, sigma, b2.bs.s, b2.bs.R, b2.K))
            bp = b2;
    }
    bool fused = false;
    bool r1_pivot = false;   // round 1 by the pivot split (pivot_round1)
    uint64_t D = 0, m = 0, G = 0;
    uint64_t seg1[3] = {0, 0, 0};
    if (bucketed) {
        bool done = false;
        rc = round1_bucketed(c, d_text, n, d_sa, bp, full_range(bp, n), s, tm, st, &done, &fused, seg1, &ksh1);
        if (rc) return rc;
        bucketed = done;
        if (done) {
            keys1 = c->keys[0];
            P = 2;
            K = bp.K;
        }
    }
    if (!bucketed) {
        const uint32_t bits1 = key_bits(base, K);
        SA_TRACE("packed: sigma=%u K=%u bits=%u", sigma, K, bits1);
        uint64_t top = 1;   // B^(K-1)
        for (uint32_t t = 1; t < K; ++t) top *= base;
        if (c->radix == 0) {
            rc = onesweep_prepare(c, s);
            if (rc) return rc;
        }
        tm.begin(SA_K_PACK);
        hipLaunchKernelGGL(k_pack_text, dim3(ch.chunks), dim3(kBlock), 0, s, d_text, n, (const uint16_t*)c->code, ch,
                           base, top, K, c->keys[1], c->hist, c->radix == 0 ? (bits1 + 7) / 8 : 0u, os_ghist(c));
        tm.end();
        SA_HIP(hipGetLastError());
        add_bytes(st, SA_K_PACK, 9 * n);
        if (c->radix == 0 && !(c->dbg & SA_DEBUG_NO_PIVOT) && n >= (1u << 16)) {
            rc = pivot_round1(c, n, bits1, d_sa, s, tm, st, &r1_pivot, &D, &m, &G, &P);
            if (rc) return rc;
        }
        if (!r1_pivot) {
            SrcKeysIota src{c->keys[1]};
            rc = radix_sort(c, src, 8 * n, ch, bits1, d_sa, c->vals_alt, c->keys[0], c->keys[1], s, tm, st, &keys1,
                            &P, true);
            if (rc) return rc;
        }
    }
    if (st) {
        st->init_chars = (int32_t)K;
        st->sigma = (int32_t)sigma;
        st->round1 = bucketed ? SA_ROUND1_BUCKETED : r1_pivot ? SA_ROUND1_PIVOT : SA_ROUND1_LSD;
    }
    int uo = 0;
    bool sparse = false;
    bool gs_ok[2] = {false, false};   // the set's group starts are in u_gs[set] (pivot rounds' MODE 1)
    if (r1_pivot) {   // pivot_round1 ran the segments (dense ranks)
        gs_ok[0] = true;
    } else if (bucketed && fused) {   // segments came with the local sort (sparse ranks)
        D = seg1[0];
        m = seg1[1];
        G = seg1[2];
        sparse = true;
    } else {
        rc = segments(c, keys1, d_sa, ch, PosIdentity{}, true, &sparse, nullptr, uo, s, tm, st, &D, &m, &G, nullptr,
                      0, RankMap{}, 0, 0, gs_buf(c, n, uo));
        if (rc) return rc;
        gs_ok[uo] = gs_buf(c, n, uo) != nullptr;
    }
    // later rounds sort in the two buffers that do not hold the round-1 keys
    uint64_t* ukb0 = keys1 == c->keys[0] ? c->keys[1] : c->keys[0];
    uint64_t* ukb1 = c->keys_u;
    const RankLookup rl{c->rank, c->member, keys1, d_text, (const uint16_t*)c->code, n, base, K,
                        bucketed ? 1u : 0u, bp.bs, bucketed ? c->segw + kBstartOff : nullptr, d_sa, ksh1};
    if (st) st->sparse_ranks = sparse ? 1 : 0;
    // the key1 samples RankLookup::sparse searches, before the first round
    // that looks a rank up through them (round 1 left them out: SegOut::samples)
    auto ensure_samples = [&]() -> int {
        if (!c->samples_pending) return SA_OK;
        c->samples_pending = false;
        const uint64_t ns = (n + (1ull << ksh1) - 1) >> ksh1;
        const uint32_t g = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((ns + kBlock - 1) / kBlock, 8192));
        tm.begin(SA_K_SORT_U);
        hipLaunchKernelGGL(k_key1_samples, dim3(g), dim3(kBlock), 0, s, d_text, n, (const uint16_t*)c->code, bp.bs,
                           (const uint32_t*)d_sa, ksh1, keys1);
        tm.end();
        SA_HIP(hipGetLastError());
        add_bytes(st, SA_K_SORT_U, 12 * ns);
        return SA_OK;
    };
    tm.round_mark();
    record_round(st, 0.f, D, P, n, K);
    SA_TRACE("  round 1: D=%llu unsorted=%llu groups=%llu", (unsigned long long)D, (unsigned long long)m,
             (unsigned long long)G);

    // doubling rounds over the unsorted set only
    const uint32_t wr = bit_width(n);   // rank values 0..n
    for (uint64_t h = K; m > 0; h *= 2) {
        if (h >= 2 * n) return set_err(SA_E_INTERNAL, "doubling did not converge (h=%llu)", (unsigned long long)h);
        const uint32_t wg = G > 1 ? bit_width(G - 1) : 0;
        const uint32_t bits = wg + wr;
        if (bits > 64) return set_err(SA_E_INTERNAL, "key of %u bits", bits);
        const Chunking cu = plan_chunks(m);
        const int ui = uo;
        uo ^= 1;
        uint64_t* sorted = nullptr;
        bool segs_done = false;   // a tied-block pivot round ran its own segments
        uint64_t Du = 0, m2 = 0, G2 = 0;
        // the first round after a bucketed round 1 with sparse ranks: the keys'
        // ranks as key1 of x + K from the text (SrcUKey1) when group id and
        // key1 + 1 fit 64 bits
        uint32_t kb1 = 0;
        if (bucketed && sparse && h == K && !(c->dbg & SA_DEBUG_NO_KEY1_ROUND)) {
            unsigned __int128 dmax = 1;
            for (uint32_t t = 0; t < bp.bs.s; ++t) dmax *= bp.bs.sigma;
            const unsigned __int128 kmax = ((dmax - 1) << bp.bs.rb) | (((unsigned __int128)1 << bp.bs.rb) - 1);
            uint32_t kw = 0;
            for (unsigned __int128 x = kmax + 1; x; x >>= 1) ++kw;
            kb1 = kw;
        }
        const bool key1_round = kb1 > 0 && kb1 + wg <= 64;
        if (c->radix == 0 && G > 0 && m <= kUsAvg * G) {
            // small groups on average: sort each group in registers, unless
            // one of them is larger than kUsLimit (then the radix sort below)
            if (sparse && !(SA_US_TWO_PHASE && key1_round)) {
                rc = ensure_samples();
                if (rc) return rc;
            }
            SA_HIP(hipMemsetAsync(c->words + kUsFlagWord, 0, 4, s));
            const uint32_t grid = (uint32_t)std::min<uint64_t>((m + kBlock - 1) / kBlock, 8192);
            tm.begin(SA_K_SORT_U);
#if SA_US_TWO_PHASE
            // the keys first, one lane per suffix, then each group's lane sorts
            // them in place (ukb0 is read and written by that lane only)
            const uint32_t gk = (uint32_t)std::min<uint64_t>((m + kBlock - 1) / kBlock, 65536);
            if (sparse && key1_round)
                hipLaunchKernelGGL(k_usort_keys<SrcUKey1>, dim3(gk), dim3(kBlock), 0, s,
                                   SrcUKey1{c->u_idx[ui], c->u_g[ui], rl, h, kb1}, m, ukb0);
            else if (sparse)
                hipLaunchKernelGGL(k_usort_keys<SrcU<true>>, dim3(gk), dim3(kBlock), 0, s,
                                   SrcU<true>{c->u_idx[ui], c->u_g[ui], rl, h, wr}, m, ukb0);
            else
                hipLaunchKernelGGL(k_usort_keys<SrcU<false>>, dim3(gk), dim3(kBlock), 0, s,
                                   SrcU<false>{c->u_idx[ui], c->u_g[ui], rl, h, wr}, m, ukb0);
            hipLaunchKernelGGL(k_usort_small<SrcKeys>, dim3(grid), dim3(kBlock), 0, s,
                               SrcKeys{ukb0, c->u_idx[ui]}, c->u_g[ui], m, ukb0, c->vals_u, c->words + kUsFlagWord);
#else
            if (sparse)
                hipLaunchKernelGGL(k_usort_small<SrcU<true>>, dim3(grid), dim3(kBlock), 0, s,
                                   SrcU<true>{c->u_idx[ui], c->u_g[ui], rl, h, wr}, c->u_g[ui], m, ukb0, c->vals_u,
                                   c->words + kUsFlagWord);
            else
                hipLaunchKernelGGL(k_usort_small<SrcU<false>>, dim3(grid), dim3(kBlock), 0, s,
                                   SrcU<false>{c->u_idx[ui], c->u_g[ui], rl, h, wr}, c->u_g[ui], m, ukb0, c->vals_u,
                                   c->words + kUsFlagWord);
#endif
            tm.end();
            SA_HIP(hipGetLastError());
            SA_HIP(hipMemcpyAsync(c->host_words + kUsFlagWord, c->words + kUsFlagWord, 4, hipMemcpyDeviceToHost, s));
            SA_HIP(host_sync(s));
            add_bytes(st, SA_K_SORT_U, 28 * m);
            if (c->host_words[kUsFlagWord] == 0) {
                sorted = ukb0;
                P = 1;
            }
            SA_TRACE("  round h=%llu: per-group register sort %s", (unsigned long long)h,
                     sorted ? "done" : "found a large group");
        }
        if (!sorted && pivot_ok(c, m, G, wr, sparse)) {
            uint64_t* kbA = ukb0 == c->keys[0] ? c->keys[1] : c->keys[0];   // the round-1 keys: dead with dense ranks
            bool gsw = false;
            rc = pivot_round(c, ui, uo, n, m, G, h, wr, ukb0, ukb1, kbA, cu, d_sa, s, tm, st, &sorted, &P,
                             &segs_done, &Du, &m2, &G2, gs_ok[ui], &gsw);
            if (rc) return rc;
            if (segs_done) gs_ok[uo] = gsw;
        }
        if (sorted) {
            rc = SA_OK;
        } else if (c->radix == 0) {
            // keys (g, rank[i + h]) once into ukb1 -- the first pass reads them
            // from there and the second overwrites them -- with the digit totals
            rc = onesweep_prepare(c, s);
            if (rc) return rc;
            const uint32_t Pu = (bits + 7) / 8;
            const uint32_t grid = (uint32_t)std::min<uint64_t>((m + kBlock - 1) / kBlock, 2048);
            if (sparse) {
                rc = ensure_samples();
                if (rc) return rc;
            }
            tm.begin(SA_K_SORT_U);
            if (sparse)
                hipLaunchKernelGGL(k_materialize<SrcU<true>>, dim3(grid), dim3(kBlock), 0, s,
                                   SrcU<true>{c->u_idx[ui], c->u_g[ui], rl, h, wr}, m, Pu, ukb1, os_ghist(c));
            else
                hipLaunchKernelGGL(k_materialize<SrcU<false>>, dim3(grid), dim3(kBlock), 0, s,
                                   SrcU<false>{c->u_idx[ui], c->u_g[ui], rl, h, wr}, m, Pu, ukb1, os_ghist(c));
            tm.end();
            SA_HIP(hipGetLastError());
            add_bytes(st, SA_K_SORT_U, 16 * m);
            rc = radix_sort(c, SrcKeys{ukb1, c->u_idx[ui]}, 12 * m, cu, bits, c->vals_u, c->vals_alt, ukb0, ukb1, s,
                            tm, st, &sorted, &P, true, true);
        } else if (sparse) {
            rc = ensure_samples();
            if (rc) return rc;
            SrcU<true> su{c->u_idx[ui], c->u_g[ui], rl, h, wr};
            rc = radix_sort(c, su, 12 * m, cu, bits, c->vals_u, c->vals_alt, ukb0, ukb1, s, tm, st, &sorted, &P,
                            false, true);
        } else {
            SrcU<false> su{c->u_idx[ui], c->u_g[ui], rl, h, wr};
            rc = radix_sort(c, su, 12 * m, cu, bits, c->vals_u, c->vals_alt, ukb0, ukb1, s, tm, st, &sorted, &P,
                            false, true);
        }
        if (rc) return rc;
        if (!segs_done) {
            rc = segments(c, sorted, c->vals_u, cu, PosArray{c->u_pos[ui]}, false, nullptr, d_sa, uo, s, tm, st, &Du,
                          &m2, &G2, nullptr, 0, RankMap{}, 0, 0, gs_buf(c, n, uo));
            if (rc) return rc;
            gs_ok[uo] = gs_buf(c, n, uo) != nullptr;
        }
        tm.round_mark();
        D = (n - m) + Du;
        record_round(st, 0.f, D, P, m, 2 * h);
        SA_TRACE("  round h=%llu: sorted %llu, D=%llu unsorted=%llu groups=%llu", (unsigned long long)h,
                 (unsigned long long)m, (unsigned long long)D, (unsigned long long)m2, (unsigned long long)G2);
        m = m2;
        G = G2;
    }
    if (D != n) return set_err(SA_E_INTERNAL, "finished with %llu groups for n=%llu", (unsigned long long)D,
                               (unsigned long long)n);
    return SA_OK;
}

static int build_device(sa_context* c, const uint8_t* d_text, uint64_t n, uint32_t* d_sa, hipStream_t s,
                        const sa_opts* opts, sa_stats* st) {
    if (st) {
        std::memset(st, 0, sizeof *st);
        st->n_kinds = SA_K_COUNT;
    }
    const int schedule = opts ? opts->schedule : SA_SCHEDULE_PACKED;
    if (st) st->schedule = schedule;
    if (n == 0) return SA_OK;
    if (!d_text || !d_sa) return set_err(SA_E_INVALID, "NULL device pointer");
    if (n > 0xFFFFFFFFull) return set_err(SA_E_INVALID, "n = %llu exceeds 2^32-1 on one device",
                                          (unsigned long long)n);
    if (schedule != SA_SCHEDULE_PACKED && schedule != SA_SCHEDULE_REFERENCE)
        return set_err(SA_E_INVALID, "unknown schedule %d", schedule);
    SA_HIP(hipSetDevice(c->device));
    int rc = ensure_capacity(c, n);
    if (rc) return rc;
    Timer tm{c, s, opts && opts->profile, st};
    c->radix = opts ? opts->radix : 0;
    set_debug(c, opts);
    if (c->radix != 0 && c->radix != 1) return set_err(SA_E_INVALID, "unknown radix algorithm %d", c->radix);
    SA_HIP(hipMemsetAsync(c->words, 0, 64, s));
    Events ev;
    rc = ev.make();
    if (rc) return rc;
    SA_TRACE("build n=%llu schedule=%d", (unsigned long long)n, schedule);
    SA_HIP(hipEventRecord(ev.e[0], s));
    if (n == 1) {
        SA_HIP(hipMemsetAsync(d_sa, 0, 4, s));
    } else if (schedule == SA_SCHEDULE_REFERENCE) {
        rc = build_reference(c, d_text, n, d_sa, s, st, tm);
    } else {
        rc = build_packed(c, d_text, n, d_sa, s, opts, st, tm);
    }
    if (rc) return rc;
    SA_HIP(hipEventRecord(ev.e[1], s));
    SA_HIP(hipEventSynchronize(ev.e[1]));
    tm.flush();
    tm.round_times();
    if (st) st->total_ms = elapsed(ev.e[0], ev.e[1]);
    return SA_OK;
}

#include "sa_dist.h"

// ---------------------------------------------------------------------------
// O(n) checker (replaces is_valid_suffix_array, manber_myers.c:184-202)
// ---------------------------------------------------------------------------
// bin shifts of a checker pass with sub-bins of 2^s2 (plan_perm's shape)
static PermPlan plan_check(uint64_t n, uint32_t s2, uint32_t b1 = 8) {
    PermPlan p;
    const uint32_t lg = bit_width(n > 1 ? n - 1 : 1);
    p.s2 = s2;
    p.s1 = std::max<uint32_t>(s2, lg > b1 ? lg - b1 : 0);
    p.nb1 = (uint32_t)((n + (1ull << p.s1) - 1) >> p.s1);
    p.nsub = 1u << (p.s1 - p.s2);
    p.tpb = (uint32_t)(((1ull << p.s1) + kPermBlock * kPermItems - 1) / (kPermBlock * kPermItems));
    return p;
}

// level-1 stripes of a permutation (sa_check.h BinStripes): `want` per bin
// when keys[0] holds the regions with their slack (2^s1 / 128, >= 2048:
// ~45 standard deviations of a stripe's fill at 1 GiB), else one
static BinStripes plan_stripes(const sa_context* c, uint64_t n, const PermPlan& p, uint32_t want) {
    BinStripes bs;
    if (want <= 1 || n < (1ull << 24)) return bs;
    const uint64_t per = ((1ull << p.s1) + want - 1) / want;
    const uint64_t scap = per + std::max<uint64_t>(2048, (1ull << p.s1) / 128);
    if ((uint64_t)p.nb1 * want * scap > c->cap_pad) return bs;
    bs.st = want;
    bs.scap = scap;
    return bs;
}

constexpr uint32_t kChkStripes = 8;   // one per XCD
constexpr uint32_t kCur2 = 1024 * kChkStripes;   // hist: level-1 cursors [stripe][bin], then level 2's

// the checker's level-1 bin bits (sa_check.h k_chk_bin NB): 8 by default;
// sa_context_set_debug's tune bits 20-23 = 1 / 2 select 10 / 9 (A/B runs)
// the checker's level-2 kernel: tune bits 20-23 = 3 take the persistent
// prefetching k_split_p (A/B runs)
static bool chk_split_persistent(const sa_context* c) { return (((uint32_t)c->tune >> 20) & 0xFu) == 3u; }

static uint32_t chk_stride(const PermPlan& p) { return p.nb1 <= 256 ? 256u : p.nb1 <= 512 ? 512u : 1024u; }

static uint32_t chk_bin_bits(const sa_context* c) {
    const uint32_t v = ((uint32_t)c->tune >> 20) & 0xFu;
    return v == 1 ? 10u : v == 2 ? 9u : 8u;
}

// Levels 1 and 2 of a permutation: (dest, value) pairs of `src` binned by
// dest (level-1 cursors per stripe and bin) and split into 2^s2-entry
// sub-bins of the final layout (keys[1], or keys[0] when s1 == s2); returns
// the pairs' buffer.  Cursors in hist (zeroed here).
template <class Src, int DSH, int TAG>
static const uint64_t* permute_levels(sa_context* c, const Src& src, uint64_t n, const PermPlan& p,
                                      const BinStripes& bs, uint32_t* err, hipStream_t s, int* rc) {
    *rc = SA_OK;
    if (hipMemsetAsync(c->hist, 0, ((uint64_t)kCur2 + (uint64_t)p.nb1 * p.nsub) * 4, s) != hipSuccess) {
        *rc = set_err(SA_E_HIP, "hipMemsetAsync failed");
        return nullptr;
    }
    const uint32_t fstride = chk_stride(p);   // cursors per stripe: k_chk_bin's NB
    if (fstride == 256) {
        constexpr uint64_t T = (uint64_t)kChkBlock * kChkItems;
        hipLaunchKernelGGL((k_chk_bin<kChkBlock, kChkItems, Src, 256>), dim3((uint32_t)((n + T - 1) / T)),
                           dim3(kChkBlock), 0, s, src, n, p.s1, c->hist, c->keys[0], err, bs);
    } else if (fstride == 512) {   // 16-bit bin tags: 7 items per lane keep two workgroups per CU
        constexpr uint64_t T = (uint64_t)kChkBlock * 7;
        hipLaunchKernelGGL((k_chk_bin<kChkBlock, 7, Src, 512>), dim3((uint32_t)((n + T - 1) / T)), dim3(kChkBlock),
                           0, s, src, n, p.s1, c->hist, c->keys[0], err, bs);
    } else {
        constexpr uint64_t T = (uint64_t)kChkBlock * 7;
        hipLaunchKernelGGL((k_chk_bin<kChkBlock, 7, Src, 1024>), dim3((uint32_t)((n + T - 1) / T)), dim3(kChkBlock),
                           0, s, src, n, p.s1, c->hist, c->keys[0], err, bs);
    }
    if (p.s1 == p.s2 && bs.st == 1) return c->keys[0];
    if (chk_split_persistent(c)) {
        uint32_t* tk = perm_tickets(c);
        if (hipMemsetAsync(tk, 0, 8 * 4, s) != hipSuccess) {
            *rc = set_err(SA_E_HIP, "hipMemsetAsync failed");
            return nullptr;
        }
        const uint32_t tpr = bs.st > 1 ? (uint32_t)((bs.scap + kPermBlock * kPermItems - 1) / (kPermBlock * kPermItems))
                                       : p.tpb;
        hipLaunchKernelGGL((k_split_p<kPermBlock, kPermItems, DSH, true, TAG>), dim3(2 * (uint32_t)c->cus),
                           dim3(kPermBlock), 0, s, (const uint64_t*)c->keys[0], n, p.s1, p.s2, p.nb1, bs.st, bs.scap,
                           tpr, (const uint32_t*)c->hist, fstride, c->hist + kCur2, c->keys[1], tk);
        return c->keys[1];
    }
    if (bs.st > 1) {
        const uint32_t tps = (uint32_t)((bs.scap + kPermBlock * kPermItems - 1) / (kPermBlock * kPermItems));
        hipLaunchKernelGGL((k_chk_split<kPermBlock, kPermItems, DSH, TAG>), dim3((p.nb1 + 7) / 8 * 8 * bs.st * tps),
                           dim3(kPermBlock), 0, s, (const uint64_t*)c->keys[0], n, p.s1, p.s2, bs, tps,
                           (const uint32_t*)c->hist, fstride, c->hist + kCur2, c->keys[1]);
    } else {
        hipLaunchKernelGGL((k_perm_split<kPermBlock, kPermItems, DSH, true, TAG>), dim3((p.nb1 + 7) / 8 * 8 * p.tpb),
                           dim3(kPermBlock), 0, s, (const uint64_t*)c->keys[0], n, p.s1, p.s2, p.tpb,
                           c->hist + kCur2, c->keys[1]);
    }
    return c->keys[1];
}

// (dest, value) pairs of `src` placed by dest into out[0, n) by the
// coalesced permutation: LCP's PHI.  Holes (0) and misplaced pairs set bits
// of *err; *err bit 128: a stripe overflowed (the caller runs it again with
// stripes = 1).
template <class Src, int TAG>
static int place_by_permutation(sa_context* c, const Src& src, uint64_t n, uint32_t* out, uint32_t* err,
                                hipStream_t s, uint32_t stripes) {
    const PermPlan p = plan_check(n, kChkSubA);
    if (p.nb1 > 256 || p.nsub > kPermMaxSub || p.s1 > 24)
        return set_err(SA_E_INTERNAL, "permutation plan out of range (n=%llu)", (unsigned long long)n);
    int rc = SA_OK;
    const uint64_t* placed = permute_levels<Src, 32, TAG>(c, src, n, p, plan_stripes(c, n, p, stripes), err, s, &rc);
    if (rc) return rc;
    hipLaunchKernelGGL((k_perm_place<kPermBlock, false, TAG>), dim3((uint32_t)((n + (1ull << kPermSub) - 1) >> kPermSub)),
                       dim3(kPermBlock), 0, s, placed, n, out, err);
    SA_HIP(hipGetLastError());
    return SA_OK;
}

// sa_check.h: pass A (ISA' by permutation) and pass B (adjacent keys compared
// in LDS per sorted sub-bin); one host sync at the end.  Workspace: ISA' in
// rank, pairs in keys[0] / keys[1], cursors in hist, sub-bin end keys in
// vals_alt.  Returns 1 valid, 0 invalid, < 0 an error.
static int check_device(sa_context* c, const uint8_t* d_text, uint64_t n, const uint32_t* d_sa, hipStream_t s) {
    if (n == 0) return 1;
    if (n > 0xFFFFFFFFull) return set_err(SA_E_INVALID, "n too large");
    if (!d_text || !d_sa) return set_err(SA_E_INVALID, "NULL device pointer");
    SA_HIP(hipSetDevice(c->device));
    int rc = ensure_capacity(c, n);
    if (rc) return rc;
    uint32_t* isa = c->rank;
    uint32_t* err = c->words + 3;
    uint32_t* cur1 = c->hist;
    uint32_t* cur2 = c->hist + kCur2;
    uint64_t* ends = reinterpret_cast<uint64_t*>(c->vals_alt);
    for (uint32_t stripes : {kChkStripes, 1u}) {
        SA_HIP(hipMemsetAsync(err, 0, 4, s));
        for (int pass = 0; pass < 2; ++pass) {
            // pass B's sub-bins: 2^13, or 2^14 once a bin would split into more
            // than the split pass's kPermMaxSub (n > 2^31)
            const uint32_t lg = bit_width(n > 1 ? n - 1 : 1);
            const uint32_t s2b = (lg > 8 && lg - 8 > kChkSubB + 10) ? kChkSubB + 1 : kChkSubB;
            const PermPlan p = plan_check(n, pass ? s2b : kChkSubA, chk_bin_bits(c));
            if (p.nb1 > 1024 || p.nsub > kPermMaxSub || p.s1 > 24)
                return set_err(SA_E_INTERNAL, "checker plan out of range (n=%llu)", (unsigned long long)n);
            const BinStripes bs = plan_stripes(c, n, p, stripes);
            const uint64_t* placed =
                pass == 0 ? permute_levels<ChkSrcA, 32, 1>(c, ChkSrcA{d_sa}, n, p, bs, err, s, &rc)
                          : permute_levels<ChkSrcB, 40, 1>(c, ChkSrcB{isa, d_text}, n, p, bs, err, s, &rc);
            if (rc) return rc;
            hipLaunchKernelGGL(k_chk_cursors,
                               dim3((uint32_t)std::min<uint64_t>(((uint64_t)p.nb1 * (p.nsub + 1) + kBlock - 1) / kBlock, 1024)),
                               dim3(kBlock), 0, s, (const uint32_t*)cur1, (const uint32_t*)cur2, n, p.s1, p.s2, p.nb1,
                               err, bs.st, chk_stride(p));
            const uint64_t nsb = (n + (1ull << p.s2) - 1) >> p.s2;
            if (pass == 0) {
                hipLaunchKernelGGL((k_perm_place<kPermBlock, false, 1>), dim3((uint32_t)nsb), dim3(kPermBlock), 0, s,
                                   placed, n, isa, err);
            } else {
                if (p.s2 == kChkSubB)
                    hipLaunchKernelGGL((k_chk_place<kChkBlock>), dim3((uint32_t)nsb), dim3(kChkBlock), 0, s, placed, n,
                                       p.s1, ends, err);
                else
                    hipLaunchKernelGGL((k_chk_place<kChkBlock, kChkSubB + 1>), dim3((uint32_t)nsb), dim3(kChkBlock), 0,
                                       s, placed, n, p.s1, ends, err);
                hipLaunchKernelGGL(k_chk_tiles, dim3((uint32_t)std::min<uint64_t>((nsb + kBlock - 1) / kBlock, 1024)),
                                   dim3(kBlock), 0, s, (const uint64_t*)ends, nsb, err);
            }
        }
        SA_HIP(hipGetLastError());
        SA_HIP(hipMemcpyAsync(c->host_words + 3, err, 4, hipMemcpyDeviceToHost, s));
        SA_HIP(host_sync(s));
        SA_TRACE("check (%u stripes): error bits %#x", stripes, c->host_words[3]);
        if (!(c->host_words[3] & 128u)) break;   // else a stripe overflowed: again with one
    }
    return c->host_words[3] == 0 ? 1 : 0;
}

// ---------------------------------------------------------------------------
// LCP + LRS (sa_lcp.h).  Workspace: PHI lives in d_lcp until the gather
// overwrites it, v / PLCP in rank, the cooperative pair lists in keys[0..1],
// their first-mismatch words in vals_alt, pair counts in counts, chunk maxima
// in hist, the LRS key in words[8..9].
// ---------------------------------------------------------------------------
static int lcp_device(sa_context* c, const uint8_t* d_text, uint64_t n, const uint32_t* d_sa, uint32_t* d_lcp,
                      uint64_t* lrs_len, uint64_t* lrs_pos, hipStream_t s) {
    if (lrs_len) *lrs_len = 0;
    if (lrs_pos) *lrs_pos = 0;
    if (n == 0) return SA_OK;
    if (!d_text || !d_sa || !d_lcp) return set_err(SA_E_INVALID, "NULL device pointer");
    if ((const void*)d_sa == (const void*)d_lcp) return set_err(SA_E_INVALID, "d_lcp may not alias d_sa");
    if (n > 0xFFFFFFFFull) return set_err(SA_E_INVALID, "n too large");
    SA_HIP(hipSetDevice(c->device));
    int rc = ensure_capacity(c, n);
    if (rc) return rc;
    uint32_t* phi = d_lcp;
    uint32_t* v = c->rank;
    uint32_t* cnt = c->counts;   // [k] = pairs in list k
    unsigned long long* best = reinterpret_cast<unsigned long long*>(c->words + 8);
    const uint32_t grid = (uint32_t)std::min<uint64_t>((n + kBlock - 1) / kBlock, 16384);
    SA_HIP(hipMemsetAsync(cnt, 0, (kLongRounds + 1) * 4, s));
    SA_HIP(hipMemsetAsync(best, 0, 8, s));
    // PHI' = PHI + 1 (0: none) by the coalesced permutation (its hole flag for
    // the smallest suffix, which has no predecessor, is expected: words[12])
    for (uint32_t stripes : {kChkStripes, 1u}) {
        SA_HIP(hipMemsetAsync(c->words + 12, 0, 4, s));
        SA_TRY(place_by_permutation<PhiSrc, 2>(c, PhiSrc{d_sa}, n, phi, c->words + 12, s, stripes));
        if (stripes == 1) break;
        // a level-1 stripe that overflowed (only an adversarial SA) lost pairs
        SA_HIP(hipMemcpyAsync(c->host_words + 12, c->words + 12, 4, hipMemcpyDeviceToHost, s));
        SA_HIP(host_sync(s));
        if (!(c->host_words[12] & 128u)) break;
    }
    hipLaunchKernelGGL(k_plcp_irreducible, dim3(grid), dim3(kBlock), 0, s, d_text, n, (const uint32_t*)phi, v,
                       c->keys[0], c->vals_alt, cnt);
    uint64_t lo = kDirect;
    for (int k = 0; k < kLongRounds && lo < n; ++k, lo *= 4) {
        const uint64_t* list = c->keys[k & 1];
        uint64_t* next = c->keys[(k + 1) & 1];
        hipLaunchKernelGGL(k_plcp_long, dim3(4096), dim3(kBlock), 0, s, d_text, n, list,
                           (const uint32_t*)(cnt + k), lo, std::min<uint64_t>(4 * lo, n), c->vals_alt);
        hipLaunchKernelGGL(k_plcp_settle, dim3(1024), dim3(kBlock), 0, s, list, (const uint32_t*)(cnt + k),
                           c->vals_alt, v, next, cnt + k + 1);
    }
    const Chunking ch = plan_chunks(n);
    hipLaunchKernelGGL(k_chunk_max, dim3(ch.chunks), dim3(kBlock), 0, s, (const uint32_t*)v, ch, c->hist);
    hipLaunchKernelGGL(k_scan_chunk_max, dim3(1), dim3(kBlock), 0, s, c->hist, ch.chunks);
    hipLaunchKernelGGL(k_plcp_apply, dim3(ch.chunks), dim3(kBlock), 0, s, v, ch, (const uint32_t*)c->hist);
    // LCP[r] = PLCP[SA[r]] (:147-155): ISA + 1 by the coalesced permutation
    // (into vals_alt, free after the long rounds), then PLCP placed at ISA
    // -- 2 x ~8.6 ms of streamed traffic at 1 GiB against a 24.7 ms random
    // 4-byte gather (146 GB moved); tune bit 30: the gather (A/B runs)
    if ((((uint32_t)c->tune >> 30) & 1u) || n < 2) {
        hipLaunchKernelGGL(k_lcp_gather, dim3(grid), dim3(kBlock), 0, s, d_sa, n, (const uint32_t*)v, d_lcp, best);
    } else {
        uint32_t* isa1 = c->vals_alt;
        for (int pass = 0; pass < 2; ++pass) {
            for (uint32_t stripes : {kChkStripes, 1u}) {
                SA_HIP(hipMemsetAsync(c->words + 12, 0, 4, s));
                if (pass == 0)
                    SA_TRY(place_by_permutation<IsaSrc, 3>(c, IsaSrc{{d_sa}}, n, isa1, c->words + 12, s, stripes));
                else
                    SA_TRY(place_by_permutation<PlcpSrc, 4>(c, PlcpSrc{isa1, v}, n, d_lcp, c->words + 12, s,
                                                            stripes));
                if (stripes == 1) break;
                SA_HIP(hipMemcpyAsync(c->host_words + 12, c->words + 12, 4, hipMemcpyDeviceToHost, s));
                SA_HIP(host_sync(s));
                if (!(c->host_words[12] & 128u)) break;
            }
        }
        hipLaunchKernelGGL(k_lcp_best, dim3(grid), dim3(kBlock), 0, s, (const uint32_t*)d_lcp, n, best);
    }
    SA_HIP(hipGetLastError());
    SA_HIP(hipMemcpyAsync(c->host_words + 8, best, 8, hipMemcpyDeviceToHost, s));
    SA_HIP(hipMemcpyAsync(c->host_words + 16, cnt, (kLongRounds + 1) * 4, hipMemcpyDeviceToHost, s));
    SA_HIP(host_sync(s));
    // every pair resolves by the last window (it reaches n); a pair left over is a bug
    uint64_t lo_end = kDirect;
    int rounds = 0;
    while (rounds < kLongRounds && lo_end < n) { lo_end *= 4; ++rounds; }
    if (c->host_words[16 + rounds] != 0)
        return set_err(SA_E_INTERNAL, "%u LCP pairs unresolved", c->host_words[16 + rounds]);
    SA_TRACE("lcp: direct-overflow pairs %u, rounds %d", c->host_words[16], rounds);
    unsigned long long b;
    std::memcpy(&b, c->host_words + 8, 8);
    const uint64_t len = b >> 32;
    if (len) {
        const uint64_t r = 0xFFFFFFFFull - (b & 0xFFFFFFFFull);
        uint32_t pos = 0;
        SA_HIP(host_memcpy(&pos, d_sa + r, 4, hipMemcpyDeviceToHost));
        if (lrs_len) *lrs_len = len;
        if (lrs_pos) *lrs_pos = pos;
    }
    return SA_OK;
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

// ---------------------------------------------------------------------------
// Host <-> HBM copies of the host-pointer entry points (the reference's
// read_file / create path, utils.c:6-48, hands over pageable malloc memory).
// Pageable copies are staged by the HIP runtime one piece at a time; here a
// ring of pinned chunks is filled by several host threads while the DMA
// engine drains the previous chunk, so the PCIe link stays busy.  Memory the
// caller already pinned (hipHostMalloc / hipHostRegister) is copied directly.
// ---------------------------------------------------------------------------
constexpr size_t kStageChunk = 32ull << 20;
constexpr int kStageBufs = 3;

static bool host_is_pinned(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// memcpy of a large block by up to 8 threads (one core moves ~10 GB/s, the
// link ~50 GB/s)
static void par_memcpy(void* dst, const void* src, size_t bytes) {
    const size_t kPiece = 4ull << 20;
    const int th = (int)std::min<size_t>(8, (bytes + kPiece - 1) / kPiece);
    if (th <= 1) {
        std::memcpy(dst, src, bytes);
        return;
    }
    std::vector<std::thread> pool;
    const size_t per = (bytes + th - 1) / th;
    for (int t = 0; t < th; ++t) {
        const size_t a = (size_t)t * per, e = std::min(bytes, a + per);
        if (a >= e) break;
        pool.emplace_back([=] { std::memcpy((char*)dst + a, (const char*)src + a, e - a); });
    }
    for (auto& x : pool) x.join();
}

struct Staging {
    void* buf[kStageBufs] = {nullptr, nullptr, nullptr};
    hipEvent_t ev[kStageBufs] = {nullptr, nullptr, nullptr};
    int make() {
        for (int i = 0; i < kStageBufs; ++i) {
            if (hipHostMalloc(&buf[i], kStageChunk, hipHostMallocDefault) != hipSuccess ||
                hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess) {
                (void)hipGetLastError();
                return set_err(SA_E_NOMEM, "pinned staging allocation failed");
            }
        }
        return SA_OK;
    }
    ~Staging() {
        for (int i = 0; i < kStageBufs; ++i) {
            if (buf[i]) hipHostFree(buf[i]);
            if (ev[i]) hipEventDestroy(ev[i]);
        }
    }
};

static int copy_h2d(void* d_dst, const void* h_src, size_t bytes, hipStream_t s) {
    if (bytes == 0) return SA_OK;
    if (bytes <= kStageChunk || host_is_pinned(h_src)) {
        SA_HIP(hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, s));
        return SA_OK;
    }
    Staging st;
    int rc = st.make();
    if (rc) return rc;
    size_t off = 0;
    for (int k = 0; off < bytes; ++k, off += kStageChunk) {
        const int b = k % kStageBufs;
        const size_t len = std::min(kStageChunk, bytes - off);
        if (k >= kStageBufs) SA_HIP(hipEventSynchronize(st.ev[b]));   // its previous DMA is done
        par_memcpy(st.buf[b], (const char*)h_src + off, len);
        SA_HIP(hipMemcpyAsync((char*)d_dst + off, st.buf[b], len, hipMemcpyHostToDevice, s));
        SA_HIP(hipEventRecord(st.ev[b], s));
    }
    SA_HIP(host_sync(s));
    return SA_OK;
}

// conv: 4 = raw u32 copy, 8 = widen u32 -> int64 into the host array
static int copy_d2h(void* h_dst, const uint32_t* d_src, uint64_t count, int width, hipStream_t s) {
    const size_t bytes = count * 4;
    if (count == 0) return SA_OK;
    if (width == 4 && (bytes <= kStageChunk || host_is_pinned(h_dst))) {
        SA_HIP(hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, s));
        SA_HIP(host_sync(s));
        return SA_OK;
    }
    Staging st;
    int rc = st.make();
    if (rc) return rc;
    const uint64_t per = kStageChunk / 4;
    const uint64_t chunks = (count + per - 1) / per;
    auto issue = [&](uint64_t k) -> int {
        const int b = (int)(k % kStageBufs);
        const uint64_t a = k * per, len = std::min(per, count - a);
        SA_HIP(hipMemcpyAsync(st.buf[b], d_src + a, len * 4, hipMemcpyDeviceToHost, s));
        SA_HIP(hipEventRecord(st.ev[b], s));
        return SA_OK;
    };
    for (uint64_t k = 0; k < chunks && k + 1 < (uint64_t)kStageBufs; ++k)
        if ((rc = issue(k))) return rc;
    for (uint64_t k = 0; k < chunks; ++k) {
        const int b = (int)(k % kStageBufs);
        SA_HIP(hipEventSynchronize(st.ev[b]));
        if (k + kStageBufs - 1 < chunks && (rc = issue(k + kStageBufs - 1))) return rc;
        const uint64_t a = k * per, len = std::min(per, count - a);
        if (width == 4) {
            par_memcpy((uint32_t*)h_dst + a, st.buf[b], len * 4);
        } else {
            const uint32_t* src = (const uint32_t*)st.buf[b];
            int64_t* o = (int64_t*)h_dst + a;
            for (uint64_t i = 0; i < len; ++i) o[i] = src[i];
        }
    }
    return SA_OK;
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

uint64_t sa_host_syncs(void) { return g_host_syncs.load(std::memory_order_relaxed); }

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
    if (hipDeviceGetAttribute(&c->cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || c->cus <= 0)
        c->cus = 256;
    if (hipMalloc(&c->hist, (size_t)kRadix * kMaxChunks * 4) != hipSuccess ||
        hipMalloc(&c->totals, kRadix * 4) != hipSuccess || hipMalloc(&c->counts, 4 * kMaxChunks * 4) != hipSuccess ||
        hipMalloc(&c->words, 64) != hipSuccess || hipMalloc(&c->alpha, 256 * 4) != hipSuccess ||
        hipMalloc(&c->code, 256 * 2) != hipSuccess ||
        hipMalloc(&c->os, (2 * kMaxPasses * kRadix + kMaxPasses) * 4) != hipSuccess ||
        hipMalloc(&c->lsd, (2 * kMaxPasses * kLsdMaxRadix + kMaxPasses) * 4 + 64) != hipSuccess ||
        hipMalloc(&c->lsdx, kLsdXqWords * 4) != hipSuccess ||
        hipMalloc(&c->segw, (kBstartOff + 2 * kBstartWords) * 4) != hipSuccess ||
        hipHostMalloc(&c->host_words, 16384, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        sa_context_destroy(c);
        return set_err(SA_E_NOMEM, "context allocation failed");
    }
    for (int i = 0; i < kEvPool + kRoundEv; ++i) {
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
    free_dist(c);
    free_ctx_buffers(c);
    free_u_buffers(c);
    hipFree(c->alpha);
    hipFree(c->code);
    hipFree(c->os);
    hipFree(c->lsd);
    hipFree(c->lsdx);
    hipFree(c->segw);
    hipFree(c->segx);
    hipFree(c->hist);
    hipFree(c->totals);
    hipFree(c->counts);
    hipFree(c->words);
    if (c->host_words) hipHostFree(c->host_words);
    for (int i = 0; i < c->ev_ready; ++i) hipEventDestroy(c->ev[i]);
    delete c;
}

int sa_context_set_debug(sa_context* ctx, const sa_opts* opts) {
    if (!ctx) return set_err(SA_E_INVALID, "NULL context");
    set_debug(ctx, opts);
    return SA_OK;
}

int sa_build_device(sa_context* ctx, const uint8_t* d_text, uint64_t n, uint32_t* d_sa, void* stream,
                    const sa_opts* opts, sa_stats* stats) {
    if (!ctx) return set_err(SA_E_INVALID, "context is NULL");
    const int rc = build_device(ctx, d_text, n, d_sa, (hipStream_t)stream, opts, stats);
    // this build's debug flags, span and launch shapes do not outlive it: a
    // later sa_dist_* build on the same context sees the defaults unless
    // sa_context_set_debug sets them again
    set_debug(ctx, nullptr);
    return rc;
}

int sa_check_device(sa_context* ctx, const uint8_t* d_text, uint64_t n, const uint32_t* d_sa, void* stream) {
    if (!ctx) return set_err(SA_E_INVALID, "context is NULL");
    return check_device(ctx, d_text, n, d_sa, (hipStream_t)stream);
}

int sa_lcp_device(sa_context* ctx, const uint8_t* d_text, uint64_t n, const uint32_t* d_sa, uint32_t* d_lcp,
                  uint64_t* lrs_len, uint64_t* lrs_pos, void* stream) {
    if (!ctx) return set_err(SA_E_INVALID, "context is NULL");
    return lcp_device(ctx, d_text, n, d_sa, d_lcp, lrs_len, lrs_pos, (hipStream_t)stream);
}

int sa_lcp(const uint8_t* text, uint64_t n, const void* sa, int sa_width, void* lcp_out, uint64_t* lrs_len,
           uint64_t* lrs_pos) {
    if (lrs_len) *lrs_len = 0;
    if (lrs_pos) *lrs_pos = 0;
    if (sa_width != 4 && sa_width != 8) return set_err(SA_E_INVALID, "sa_width must be 4 or 8");
    if (n == 0) return SA_OK;
    if (!text || !sa || !lcp_out) return set_err(SA_E_INVALID, "NULL host pointer");
    if (n > 0xFFFFFFFFull) return set_err(SA_E_INVALID, "n too large");
    std::vector<uint32_t> narrow;
    const void* src = sa;
    if (sa_width == 8) {
        narrow.resize(n);
        const int64_t* w = (const int64_t*)sa;
        for (uint64_t i = 0; i < n; ++i) {
            if (w[i] < 0 || (uint64_t)w[i] >= n) return set_err(SA_E_INVALID, "SA entry out of range");
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
    uint32_t* d_lcp = nullptr;
    if (hipMalloc(&d_text, align_up(n, 256)) != hipSuccess || hipMalloc(&d_sa, align_up(n, 64) * 4) != hipSuccess ||
        hipMalloc(&d_lcp, align_up(n, 64) * 4) != hipSuccess) {
        hipFree(d_text);
        hipFree(d_sa);
        (void)hipGetLastError();
        return set_err(SA_E_NOMEM, "device allocation failed");
    }
    if (copy_h2d(d_text, text, n, nullptr) != SA_OK || copy_h2d(d_sa, src, n * 4, nullptr) != SA_OK ||
        host_sync(nullptr) != hipSuccess)
        rc = set_err(SA_E_HIP, "H2D copy failed: %s", g_err.c_str());
    // the checker rejects a non-permutation before PHI would scatter through it
    if (rc == SA_OK) {
        rc = check_device(c, d_text, n, d_sa, nullptr);
        if (rc == 0) rc = set_err(SA_E_INVALID, "not a valid suffix array of the text");
        else if (rc == 1) rc = SA_OK;
    }
    if (rc == SA_OK) rc = lcp_device(c, d_text, n, d_sa, d_lcp, lrs_len, lrs_pos, nullptr);
    if (rc == SA_OK) {
        rc = copy_d2h(lcp_out, d_lcp, n, sa_width, nullptr);
    }
    hipFree(d_text);
    hipFree(d_sa);
    hipFree(d_lcp);
    return rc;
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
    // PCIe legs timed on the host clock (pinned staging overlaps host copies
    // with the DMA; sa_stats reports them apart from total_ms)
    auto t0 = std::chrono::steady_clock::now();
    rc = copy_h2d(d_text, text, n, s);
    if (rc == SA_OK) SA_HIP(host_sync(s));
    auto t1 = std::chrono::steady_clock::now();
    const double h2d = std::chrono::duration<double, std::milli>(t1 - t0).count();
    if (rc == SA_OK) rc = build_device(c, d_text, n, d_sa, s, opts, stats);
    double d2h = 0.0;
    if (rc == SA_OK) {
        t0 = std::chrono::steady_clock::now();
        rc = copy_d2h(sa_out, d_sa, n, sa_width, s);
        d2h = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    if (stats) {
        stats->h2d_ms = h2d;
        stats->d2h_ms = d2h;
    }
    hipFree(d_text);
    hipFree(d_sa);
    return rc;
}

// dst[idx[i] - base] = src[i]; indices outside [base, base + dst_n) are
// skipped and counted (the host turns a non-zero count into an error).
__global__ __launch_bounds__(256) void k_scatter_u64(uint64_t* __restrict__ dst, uint64_t dst_n,
                                                     const int64_t* __restrict__ idx, int64_t base,
                                                     const uint64_t* __restrict__ src, uint64_t m,
                                                     unsigned long long* __restrict__ bad) {
    uint32_t nbad = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t j = (uint64_t)(idx[i] - base);
        if (j < dst_n) dst[j] = src[i];
        else ++nbad;
    }
    if (nbad) atomicAdd(bad, (unsigned long long)nbad);
}

int sa_scatter_u64_device(uint64_t* d_dst, uint64_t dst_n, const int64_t* d_idx, int64_t base,
                          const uint64_t* d_src, uint64_t m, void* stream) {
    if (m == 0) return SA_OK;
    if (!d_dst || !d_idx || !d_src) return set_err(SA_E_INVALID, "NULL device pointer");
    hipStream_t s = (hipStream_t)stream;
    unsigned long long* d_bad = nullptr;
    unsigned long long bad = 0;
    SA_HIP(hipMallocAsync((void**)&d_bad, 8, s));
    SA_HIP(hipMemsetAsync(d_bad, 0, 8, s));
    const uint32_t grid = (uint32_t)std::min<uint64_t>((m + 255) / 256, 8192);
    hipLaunchKernelGGL(k_scatter_u64, dim3(grid), dim3(256), 0, s, d_dst, dst_n, d_idx, base, d_src, m, d_bad);
    SA_HIP(hipGetLastError());
    SA_HIP(hipMemcpyAsync(&bad, d_bad, 8, hipMemcpyDeviceToHost, s));
    SA_HIP(hipFreeAsync(d_bad, s));
    SA_HIP(host_sync(s));
    if (bad) return set_err(SA_E_INVALID, "%llu scatter indices outside [%lld, %lld)", bad, (long long)base,
                            (long long)(base + (int64_t)dst_n));
    return SA_OK;
}

// dst[i] = src[idx[i] - base]; out-of-range indices write 0 and are counted.
__global__ __launch_bounds__(256) void k_gather_u64(uint64_t* __restrict__ dst, const uint64_t* __restrict__ src,
                                                    uint64_t src_n, const int64_t* __restrict__ idx, int64_t base,
                                                    uint64_t m, unsigned long long* __restrict__ bad) {
    uint32_t nbad = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t j = (uint64_t)(idx[i] - base);
        uint64_t v = 0;
        if (j < src_n) v = src[j];
        else ++nbad;
        dst[i] = v;
    }
    if (nbad) atomicAdd(bad, (unsigned long long)nbad);
}

int sa_gather_u64_device(uint64_t* d_dst, const uint64_t* d_src, uint64_t src_n, const int64_t* d_idx, int64_t base,
                         uint64_t m, void* stream) {
    if (m == 0) return SA_OK;
    if (!d_dst || !d_idx || !d_src) return set_err(SA_E_INVALID, "NULL device pointer");
    hipStream_t s = (hipStream_t)stream;
    unsigned long long* d_bad = nullptr;
    unsigned long long bad = 0;
    SA_HIP(hipMallocAsync((void**)&d_bad, 8, s));
    SA_HIP(hipMemsetAsync(d_bad, 0, 8, s));
    const uint32_t grid = (uint32_t)std::min<uint64_t>((m + 255) / 256, 8192);
    hipLaunchKernelGGL(k_gather_u64, dim3(grid), dim3(256), 0, s, d_dst, d_src, src_n, d_idx, base, m, d_bad);
    SA_HIP(hipGetLastError());
    SA_HIP(hipMemcpyAsync(&bad, d_bad, 8, hipMemcpyDeviceToHost, s));
    SA_HIP(hipFreeAsync(d_bad, s));
    SA_HIP(host_sync(s));
    if (bad) return set_err(SA_E_INVALID, "%llu gather indices outside [%lld, %lld)", bad, (long long)base,
                            (long long)(base + (int64_t)src_n));
    return SA_OK;
}

}  // extern "C"

// Inclusive scans of m int64 values in place (running max: the group-start
// carries of the sample-sort driver; sum: its dense group ids): per-tile
// totals (256 lanes x 16 contiguous values), one workgroup scans the tile
// totals, each tile then scans itself from its carry.
constexpr int kRmBlock = 256, kRmItems = 16, kRmTile = kRmBlock * kRmItems;

struct ScanMax {
    static __device__ __forceinline__ int64_t id() { return INT64_MIN; }
    static __device__ __forceinline__ int64_t f(int64_t a, int64_t b) { return a > b ? a : b; }
};
struct ScanSum {
    static __device__ __forceinline__ int64_t id() { return 0; }
    static __device__ __forceinline__ int64_t f(int64_t a, int64_t b) { return a + b; }
};

template <class Op>
__device__ inline int64_t rm_block_incl(int64_t v, int64_t* s_w) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(v, o, 64);
        if (lane >= o) v = Op::f(y, v);
    }
    if (lane == 63) s_w[w] = v;
    __syncthreads();
    int64_t c = Op::id();
    for (int q = 0; q < w; ++q) c = Op::f(c, s_w[q]);
    return Op::f(c, v);
}

// exclusive block scan: the inclusive value of the previous lane
template <class Op>
__device__ inline int64_t rm_block_excl(int64_t v, int64_t* s_w) {
    const int64_t incl = rm_block_incl<Op>(v, s_w);
    int64_t c = __shfl_up(incl, 1, 64);
    if ((threadIdx.x & 63) == 0) {
        c = Op::id();
        for (int q = 0; q < (int)(threadIdx.x >> 6); ++q) c = Op::f(c, s_w[q]);
    }
    return c;
}

template <class Op>
__global__ __launch_bounds__(kRmBlock) void k_rmax_tiles(const int64_t* __restrict__ v, uint64_t m,
                                                         int64_t* __restrict__ tmax) {
    __shared__ int64_t s_w[kRmBlock / 64];
    const uint64_t b0 = (uint64_t)blockIdx.x * kRmTile + (uint64_t)threadIdx.x * kRmItems;
    int64_t x = Op::id();
    for (int j = 0; j < kRmItems; ++j)
        if (b0 + j < m) x = Op::f(x, v[b0 + j]);
    x = rm_block_incl<Op>(x, s_w);
    if (threadIdx.x == kRmBlock - 1) tmax[blockIdx.x] = x;
}

// exclusive scan of the tile totals (one workgroup of kRmBlock lanes); the
// grand total lands in tmax[tiles]
template <class Op>
__global__ __launch_bounds__(kRmBlock) void k_rmax_carry(int64_t* __restrict__ tmax, uint64_t tiles) {
    __shared__ int64_t s_w[kRmBlock / 64];
    const uint64_t per = (tiles + kRmBlock - 1) / kRmBlock;
    const uint64_t a = (uint64_t)threadIdx.x * per, e = a + per < tiles ? a + per : tiles;
    int64_t x = Op::id();
    for (uint64_t i = a; i < e; ++i) x = Op::f(x, tmax[i]);
    int64_t c = rm_block_excl<Op>(x, s_w);
    for (uint64_t i = a; i < e; ++i) {
        const int64_t y = tmax[i];
        tmax[i] = c;
        c = Op::f(c, y);
    }
    if (a < tiles && e == tiles) tmax[tiles] = c;
}

template <class Op>
__global__ __launch_bounds__(kRmBlock) void k_rmax_apply(int64_t* __restrict__ v, uint64_t m,
                                                         const int64_t* __restrict__ tcarry) {
    __shared__ int64_t s_w[kRmBlock / 64];
    const uint64_t b0 = (uint64_t)blockIdx.x * kRmTile + (uint64_t)threadIdx.x * kRmItems;
    int64_t r[kRmItems];
    int64_t x = Op::id();
    for (int j = 0; j < kRmItems; ++j) {
        r[j] = b0 + j < m ? v[b0 + j] : Op::id();
        x = Op::f(x, r[j]);
    }
    int64_t c = Op::f(tcarry[blockIdx.x], rm_block_excl<Op>(x, s_w));
    for (int j = 0; j < kRmItems; ++j) {
        c = Op::f(c, r[j]);
        if (b0 + j < m) v[b0 + j] = c;
    }
}




// out[i] = #{ j : sorted[j] < q[i] } (<= with RIGHT): one lane per query
template <bool RIGHT>
__global__ __launch_bounds__(kBlock) void k_count_below(const uint64_t* __restrict__ sorted, uint64_t m,
                                                        const uint64_t* __restrict__ q, uint64_t nq,
                                                        int64_t* __restrict__ out) {
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < nq; i += (uint64_t)gridDim.x * kBlock) {
        const uint64_t x = q[i];
        uint64_t lo = 0, hi = m;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) / 2;
            if (RIGHT ? sorted[mid] <= x : sorted[mid] < x) lo = mid + 1;
            else hi = mid;
        }
        out[i] = (int64_t)lo;
    }
}


// Stream compaction of a byte mask: per-tile counts of the non-zero bytes
// (16 per lane), their exclusive sum (k_rmax_carry<ScanSum>), then each tile
// writes its positions in order.
__global__ __launch_bounds__(kRmBlock) void k_sel_count(const uint8_t* __restrict__ mask, uint64_t m,
                                                        int64_t* __restrict__ tcnt) {
    __shared__ int64_t s_w[kRmBlock / 64];
    const uint64_t b0 = (uint64_t)blockIdx.x * kRmTile + (uint64_t)threadIdx.x * kRmItems;
    int64_t c = 0;
    for (int j = 0; j < kRmItems; ++j) c += (b0 + j < m && mask[b0 + j]) ? 1 : 0;
    c = rm_block_incl<ScanSum>(c, s_w);
    if (threadIdx.x == kRmBlock - 1) tcnt[blockIdx.x] = c;
}

__global__ __launch_bounds__(kRmBlock) void k_sel_write(const uint8_t* __restrict__ mask, uint64_t m,
                                                        const int64_t* __restrict__ toff, int64_t* __restrict__ out) {
    __shared__ int64_t s_w[kRmBlock / 64];
    const uint64_t b0 = (uint64_t)blockIdx.x * kRmTile + (uint64_t)threadIdx.x * kRmItems;
    uint32_t bits = 0;
    for (int j = 0; j < kRmItems; ++j) bits |= (b0 + j < m && mask[b0 + j]) ? 1u << j : 0u;
    int64_t o = toff[blockIdx.x] + rm_block_excl<ScanSum>((int64_t)__popc(bits), s_w);
    while (bits) {
        const int j = __builtin_ctz(bits);
        bits &= bits - 1u;
        out[o++] = (int64_t)(b0 + j);
    }
}

template <class Op>
static int scan_i64(int64_t* d_v, uint64_t m, hipStream_t s) {
    const uint64_t tiles = (m + kRmTile - 1) / kRmTile;
    if (tiles > 0xFFFFFFFFull) return set_err(SA_E_INVALID, "m too large");
    int64_t* d_t = nullptr;
    SA_HIP(hipMallocAsync((void**)&d_t, (tiles + 1) * 8, s));
    hipLaunchKernelGGL(k_rmax_tiles<Op>, dim3((uint32_t)tiles), dim3(kRmBlock), 0, s, d_v, m, d_t);
    hipLaunchKernelGGL(k_rmax_carry<Op>, dim3(1), dim3(kRmBlock), 0, s, d_t, tiles);
    hipLaunchKernelGGL(k_rmax_apply<Op>, dim3((uint32_t)tiles), dim3(kRmBlock), 0, s, d_v, m, d_t);
    SA_HIP(hipGetLastError());
    SA_HIP(hipFreeAsync(d_t, s));
    return SA_OK;
}

extern "C" {

int sa_running_max_i64_device(int64_t* d_v, uint64_t m, void* stream) {
    if (m == 0) return SA_OK;
    if (!d_v) return set_err(SA_E_INVALID, "NULL device pointer");
    return scan_i64<ScanMax>(d_v, m, (hipStream_t)stream);
}

int sa_inclusive_sum_i64_device(int64_t* d_v, uint64_t m, void* stream) {
    if (m == 0) return SA_OK;
    if (!d_v) return set_err(SA_E_INVALID, "NULL device pointer");
    return scan_i64<ScanSum>(d_v, m, (hipStream_t)stream);
}

int sa_count_below_u64_device(const uint64_t* d_sorted, uint64_t m, const uint64_t* d_q, uint64_t nq, int right,
                              int64_t* d_out, void* stream) {
    if (nq == 0) return SA_OK;
    if ((!d_sorted && m) || !d_q || !d_out) return set_err(SA_E_INVALID, "NULL device pointer");
    hipStream_t s = (hipStream_t)stream;
    const uint32_t grid = (uint32_t)std::min<uint64_t>((nq + kBlock - 1) / kBlock, 8192);
    if (right) hipLaunchKernelGGL(k_count_below<true>, dim3(grid), dim3(kBlock), 0, s, d_sorted, m, d_q, nq, d_out);
    else hipLaunchKernelGGL(k_count_below<false>, dim3(grid), dim3(kBlock), 0, s, d_sorted, m, d_q, nq, d_out);
    SA_HIP(hipGetLastError());
    return SA_OK;
}

int sa_select_u8_device(const uint8_t* d_mask, uint64_t m, int64_t* d_out, uint64_t* count, void* stream) {
    if (!count) return set_err(SA_E_INVALID, "count is NULL");
    *count = 0;
    if (m == 0) return SA_OK;
    if (!d_mask) return set_err(SA_E_INVALID, "NULL device pointer");
    hipStream_t s = (hipStream_t)stream;
    const uint64_t tiles = (m + kRmTile - 1) / kRmTile;
    if (tiles > 0xFFFFFFFFull) return set_err(SA_E_INVALID, "m too large");
    int64_t* d_t = nullptr;
    int64_t total = 0;
    SA_HIP(hipMallocAsync((void**)&d_t, (tiles + 1) * 8, s));
    hipLaunchKernelGGL(k_sel_count, dim3((uint32_t)tiles), dim3(kRmBlock), 0, s, d_mask, m, d_t);
    hipLaunchKernelGGL(k_rmax_carry<ScanSum>, dim3(1), dim3(kRmBlock), 0, s, d_t, tiles);
    if (d_out) hipLaunchKernelGGL(k_sel_write, dim3((uint32_t)tiles), dim3(kRmBlock), 0, s, d_mask, m, d_t, d_out);
    SA_HIP(hipGetLastError());
    SA_HIP(hipMemcpyAsync(&total, d_t + tiles, 8, hipMemcpyDeviceToHost, s));
    SA_HIP(hipFreeAsync(d_t, s));
    SA_HIP(host_sync(s));
    *count = (uint64_t)total;
    return SA_OK;
}

int sa_alphabet_device(const uint8_t* d_text, uint64_t n, uint32_t present_out[8], void* stream) {
    if (!present_out) return set_err(SA_E_INVALID, "present_out is NULL");
    std::memset(present_out, 0, 32);
    if (n == 0) return SA_OK;
    if (!d_text) return set_err(SA_E_INVALID, "NULL device pointer");
    hipStream_t s = (hipStream_t)stream;
    uint32_t* d_mask = nullptr;
    SA_HIP(hipMallocAsync((void**)&d_mask, 32, s));
    SA_HIP(hipMemsetAsync(d_mask, 0, 32, s));
    const uint32_t grid = (uint32_t)std::min<uint64_t>((n + kBlock * 16 - 1) / (kBlock * 16), 2048);
    hipLaunchKernelGGL(k_alphabet, dim3(grid), dim3(kBlock), 0, s, d_text, n, d_mask);
    SA_HIP(hipGetLastError());
    SA_HIP(hipMemcpyAsync(present_out, d_mask, 32, hipMemcpyDeviceToHost, s));
    SA_HIP(hipFreeAsync(d_mask, s));
    SA_HIP(host_sync(s));
    return SA_OK;
}

int sa_pack_keys_device(sa_context* ctx, const uint8_t* d_text, uint64_t n, uint64_t lo, uint64_t hi,
                        const uint16_t code[256], uint64_t base, uint32_t K, uint64_t* d_keys_out, void* stream) {
    if (lo > hi || hi > n) return set_err(SA_E_INVALID, "bad range [%llu, %llu) of %llu", (unsigned long long)lo,
                                          (unsigned long long)hi, (unsigned long long)n);
    if (K == 0 || K >= (uint32_t)kMaxK || base < 2 || key_bits(base, K) > 64)
        return set_err(SA_E_INVALID, "bad packing K=%u base=%llu", K, (unsigned long long)base);
    // an empty slice (n < world size) writes nothing: a zero-element tensor's
    // data pointer may be NULL
    if (hi == lo) return SA_OK;
    if (!ctx || !d_text || !d_keys_out || !code) return set_err(SA_E_INVALID, "NULL argument");
    hipStream_t s = (hipStream_t)stream;
    SA_HIP(hipSetDevice(ctx->device));
    // the caller's code[] may be a temporary: stage it in the context's pinned
    // words and wait for the copy before returning
    uint16_t* h_code = reinterpret_cast<uint16_t*>(ctx->host_words + 320);
    std::memcpy(h_code, code, 512);
    SA_HIP(hipMemcpyAsync(ctx->code, h_code, 512, hipMemcpyHostToDevice, s));
    SA_HIP(host_sync(s));
    uint64_t top = 1;
    for (uint32_t t = 1; t < K; ++t) top *= base;
    const Chunking ch = plan_chunks(hi - lo);
    hipLaunchKernelGGL(k_pack_text, dim3(ch.chunks), dim3(kBlock), 0, s, d_text + lo, n - lo,
                       (const uint16_t*)ctx->code, ch, base, top, K, d_keys_out, (uint32_t*)nullptr, 0u,
                       (uint32_t*)nullptr);
    SA_HIP(hipGetLastError());
    return SA_OK;
}

int sa_sort_pairs_device(sa_context* ctx, const uint64_t* d_keys_in, const uint32_t* d_vals_in, uint64_t m,
                         uint32_t bits, uint64_t* d_keys_out, uint32_t* d_vals_out, void* stream) {
    if (!ctx || !d_keys_in || !d_vals_in || !d_keys_out || !d_vals_out) return set_err(SA_E_INVALID, "NULL argument");
    if (bits == 0 || bits > 64) return set_err(SA_E_INVALID, "bits must be 1..64");
    if (m == 0) return SA_OK;
    if (m > 0xFFFFFFFFull) return set_err(SA_E_INVALID, "m too large");
    if ((const void*)d_keys_in == (const void*)d_keys_out || (const void*)d_vals_in == (const void*)d_vals_out)
        return set_err(SA_E_INVALID, "outputs may not alias inputs");
    hipStream_t s = (hipStream_t)stream;
    SA_HIP(hipSetDevice(ctx->device));
    int rc = ensure_capacity(ctx, m);
    if (rc) return rc;
    ctx->radix = 0;
    SA_HIP(hipMemsetAsync(ctx->words, 0, 64, s));
    Timer tm{ctx, s, false, nullptr};
    const Chunking ch = plan_chunks(m);
    SrcKeys src{d_keys_in, d_vals_in};
    uint64_t* sorted;
    uint32_t P;
    rc = radix_sort(ctx, src, 12 * m, ch, bits, d_vals_out, ctx->vals_alt, d_keys_out, ctx->keys[1], s, tm, nullptr,
                    &sorted, &P);
    if (rc) return rc;
    if (sorted != d_keys_out) SA_HIP(hipMemcpyAsync(d_keys_out, sorted, m * 8, hipMemcpyDeviceToDevice, s));
    SA_HIP(hipMemcpyAsync(ctx->host_words, ctx->words, 20, hipMemcpyDeviceToHost, s));
    SA_HIP(host_sync(s));
    if (ctx->host_words[4]) return set_err(SA_E_INTERNAL, "radix look-back did not complete");
    return SA_OK;
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

// ---- range-partitioned multi-GPU build (sa_dist.h) ----------------------
int sa_dist_begin(sa_context* ctx, const uint8_t* d_text, uint64_t n, int world, int rank,
                  const uint32_t present[8], uint64_t* d_coarse, void* stream, sa_dist_info* info) {
    if (!ctx || !info) return set_err(SA_E_INVALID, "NULL argument");
    return dist_begin(ctx, d_text, n, world, rank, present, d_coarse, (hipStream_t)stream, info);
}

int sa_dist_cuts(sa_context* ctx, const uint64_t* h_coarse, sa_dist_info* info) {
    if (!ctx || !info) return set_err(SA_E_INVALID, "NULL argument");
    return dist_cuts(ctx, h_coarse, info);
}

int sa_dist_reserve(sa_context* ctx, uint64_t max_n, int world) {
    if (!ctx) return set_err(SA_E_INVALID, "NULL argument");
    return dist_reserve(ctx, max_n, world);
}

int sa_dist_release(sa_context* ctx) {
    if (!ctx) return set_err(SA_E_INVALID, "NULL argument");
    SA_HIP(hipSetDevice(ctx->device));
    SA_HIP(hipDeviceSynchronize());
    free_dist(ctx);
    return SA_OK;
}

int sa_dist_plan_cuts(int world, uint64_t n, int bucket_bits, const uint64_t* h_coarse, uint32_t* cuts_out,
                      uint64_t* m_max) {
    if (world < 1 || world > kDistMaxWorld || !h_coarse || !cuts_out || !m_max)
        return set_err(SA_E_INVALID, "bad argument");
    if (bucket_bits < (int)kCoarseBits || bucket_bits > 32) return set_err(SA_E_INVALID, "bucket_bits out of range");
    std::vector<uint64_t> pre(kCoarse + 1, 0);
    for (uint32_t i = 0; i < kCoarse; ++i) pre[i + 1] = pre[i] + h_coarse[i];
    if (pre[kCoarse] != n) return set_err(SA_E_INVALID, "coarse histogram does not sum to n");
    return plan_cuts(world, n, (uint32_t)bucket_bits - kCoarseBits, pre.data(), cuts_out, m_max) ? SA_DIST_OK
                                                                                                  : SA_DIST_UNBALANCED;
}

int sa_dist_round1(sa_context* ctx, uint32_t* d_sa_local, void* stream, sa_dist_info* info, sa_stats* stats) {
    if (!ctx || !info) return set_err(SA_E_INVALID, "NULL argument");
    if (!ctx->dist) return set_err(SA_E_INVALID, "sa_dist_round1 before sa_dist_begin");
    return dist_round1(ctx, ctx->dist->text, d_sa_local, (hipStream_t)stream, info, stats);
}

int sa_dist_req_count(sa_context* ctx, uint64_t h, uint64_t* counts_out, void* stream, sa_dist_info* info) {
    if (!ctx || !counts_out || !info) return set_err(SA_E_INVALID, "NULL argument");
    return dist_req_count(ctx, h, counts_out, (hipStream_t)stream, info);
}

int sa_dist_req_fill(sa_context* ctx, uint64_t h, uint32_t* d_req, void* stream) {
    if (!ctx) return set_err(SA_E_INVALID, "NULL argument");
    return dist_req_fill(ctx, h, d_req, (hipStream_t)stream);
}

int sa_dist_answer(sa_context* ctx, const uint32_t* d_req, uint64_t nreq, uint64_t* d_ans, void* stream) {
    if (!ctx) return set_err(SA_E_INVALID, "NULL argument");
    return dist_answer(ctx, d_req, nreq, d_ans, (hipStream_t)stream);
}

int sa_dist_refine(sa_context* ctx, uint64_t h, const uint64_t* d_ans, uint32_t* d_sa_local, void* stream,
                   sa_dist_info* info) {
    if (!ctx || !info) return set_err(SA_E_INVALID, "NULL argument");
    return dist_refine(ctx, h, d_ans, d_sa_local, (hipStream_t)stream, info);
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
    if (copy_h2d(d_text, text, n, nullptr) != SA_OK || copy_h2d(d_sa, src, n * 4, nullptr) != SA_OK ||
        host_sync(nullptr) != hipSuccess)
        rc = set_err(SA_E_HIP, "H2D copy failed: %s", g_err.c_str());
    if (rc == SA_OK) rc = check_device(c, d_text, n, d_sa, nullptr);
    hipFree(d_text);
    hipFree(d_sa);
    return rc;
}

}  // extern "C"
