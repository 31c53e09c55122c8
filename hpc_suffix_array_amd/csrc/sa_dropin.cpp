// sa_dropin.cpp -- the six drop-in symbols of include/suffix_array.h
// (reference: src/common/suffix_array.h:24-29, src/sequential/manber_myers.c).
//
// build_suffix_array and is_valid_suffix_array run on the GPU through the
// extended ABI (sa_build_ex / sa_check).  There is no CPU fallback: on any
// failure the reason is printed to stderr and the process aborts, the same
// contract as the reference's assert on allocation failure (manber_myers.c:85).
// build_lcp_array runs on the GPU too (sa_lcp); find_longest_repeated_substring
// keeps the reference's O(n) scan of the caller's lcp array (manber_myers.c:
// 159-182) -- the device path reports the same answer from sa_lcp_device.
#include <cstddef>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/sa_hip.h"
#include "../../include/suffix_array.h"

static_assert(sizeof(SuffixArray) == 32, "SuffixArray must keep the reference's 32-byte layout");
static_assert(offsetof(SuffixArray, n) == 8 && offsetof(SuffixArray, sa) == 16 && offsetof(SuffixArray, lcp) == 24,
              "SuffixArray field offsets must match suffix_array.h:16-21");

[[noreturn]] static void die(const char* what) {
    std::fprintf(stderr, "libsa_hip: %s failed: %s\n", what, sa_last_error());
    std::abort();
}

extern "C" {

// manber_myers.c:51-69: private copy with strncpy semantics (bytes after the
// first NUL are NUL), plus malloc'd sa and lcp arrays; NULL on failure.
SuffixArray* create_suffix_array(const char* S, int n) {
    if (n < 0) return nullptr;
    SuffixArray* sa = (SuffixArray*)std::malloc(sizeof(SuffixArray));
    if (!sa) return nullptr;
    sa->n = n;
    sa->str = (char*)std::malloc((size_t)n + 1);
    if (!sa->str) {
        std::free(sa);
        return nullptr;
    }
    std::strncpy(sa->str, S ? S : "", (size_t)n);
    sa->str[n] = '\0';
    sa->sa = (int*)std::malloc((size_t)(n ? n : 1) * sizeof(int));
    sa->lcp = (int*)std::malloc((size_t)(n ? n : 1) * sizeof(int));
    if (!sa->sa || !sa->lcp) {
        std::free(sa->str);
        std::free(sa->sa);
        std::free(sa->lcp);
        std::free(sa);
        return nullptr;
    }
    return sa;
}

void destroy_suffix_array(SuffixArray* sa) {
    if (!sa) return;
    std::free(sa->str);
    std::free(sa->sa);
    std::free(sa->lcp);
    std::free(sa);
}

void build_suffix_array(SuffixArray* sa) {
    if (!sa || sa->n <= 0) return;
    if (sa_build_ex((const uint8_t*)sa->str, (uint64_t)sa->n, sa->sa, 4, nullptr, nullptr) != SA_OK)
        die("build_suffix_array");
}

// manber_myers.c:135-157 on the GPU (sa_lcp: PHI / irreducible-LCP method,
// the values of the reference's Kasai loop); lcp[0] = 0.
void build_lcp_array(SuffixArray* sa) {
    if (!sa || sa->n <= 0) return;
    if (sa_lcp((const uint8_t*)sa->str, (uint64_t)sa->n, sa->sa, 4, sa->lcp, nullptr, nullptr) != SA_OK)
        die("build_lcp_array");
}

// manber_myers.c:159-182: first position of the strictly largest LCP.
char* find_longest_repeated_substring(SuffixArray* sa) {
    if (!sa || !sa->lcp) return nullptr;
    int best = 0, at = -1;
    for (int r = 1; r < sa->n; ++r)
        if (sa->lcp[r] > best) {
            best = sa->lcp[r];
            at = r;
        }
    if (best == 0) return nullptr;
    char* out = (char*)std::malloc((size_t)best + 1);
    if (!out) return nullptr;
    std::strncpy(out, sa->str + sa->sa[at], (size_t)best);
    out[best] = '\0';
    return out;
}

int is_valid_suffix_array(SuffixArray* sa) {
    if (!sa || sa->n <= 0) return 1;
    const int r = sa_check((const uint8_t*)sa->str, (uint64_t)sa->n, sa->sa, 4);
    if (r < 0) die("is_valid_suffix_array");
    return r;
}

}  // extern "C"

extern "C" uint64_t sa_struct_size(int which) {
    return which == 0 ? sizeof(sa_stats) : which == 1 ? sizeof(sa_opts) : 0;
}
