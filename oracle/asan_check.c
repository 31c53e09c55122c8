/*
 * oracle/asan_check.c -- TEST INFRASTRUCTURE: drives the C restatement
 * (mm_oracle.c) under AddressSanitizer + UndefinedBehaviorSanitizer on the
 * edge cases the reference's own tests exercise (empty,
 * one symbol, degenerate runs, byte values 0x00 and 0xFF, ragged sizes) and
 * checks every result with the restatement's O(n) checker and Kasai LCP.
 * Built by `make -C oracle asan` (host code only), run by
 * tests/test_oracle.py::test_oracle_under_sanitizers.  Exit status 0 = clean.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int oracle_build_sa(const uint8_t* text, uint64_t n, uint32_t* sa_out, double* round_ms, uint64_t* distinct,
                    int max_rounds);
int oracle_lcp(const uint8_t* text, uint64_t n, const uint32_t* sa, uint32_t* lcp);
uint64_t oracle_lrs(uint64_t n, const uint32_t* sa, const uint32_t* lcp, uint64_t* pos);
int oracle_check_sa(const uint8_t* text, uint64_t n, const uint32_t* sa);
void oracle_gen_text(uint8_t* out, uint64_t n, uint64_t seed, const uint8_t* alpha, uint32_t sigma);

static int run(const char* name, const uint8_t* t, uint64_t n) {
    uint32_t* sa = malloc((n ? n : 1) * sizeof *sa);
    uint32_t* lcp = malloc((n ? n : 1) * sizeof *lcp);
    double rs[64];
    uint64_t dj[64];
    int bad = 0;
    const int rounds = oracle_build_sa(t, n, sa, rs, dj, 64);
    if (rounds < 0) bad = 1;
    else if (n && oracle_check_sa(t, n, sa) != 1) bad = 2;
    else if (n && oracle_lcp(t, n, sa, lcp) != 0) bad = 3;
    if (!bad && n) {
        uint64_t pos = 0;
        (void)oracle_lrs(n, sa, lcp, &pos);
    }
    printf("%-28s n=%-8llu rounds=%-3d %s\n", name, (unsigned long long)n, rounds, bad ? "FAIL" : "ok");
    free(sa);
    free(lcp);
    return bad;
}

int main(void) {
    int bad = 0;
    static const uint8_t dna[] = "ACGT", bin[] = "ab";
    uint8_t all[256];
    for (int i = 0; i < 256; ++i) all[i] = (uint8_t)i;
    bad |= run("empty", (const uint8_t*)"", 0);
    bad |= run("one symbol", (const uint8_t*)"x", 1);
    bad |= run("banana", (const uint8_t*)"banana", 6);
    uint8_t* t = malloc(1 << 20);
    memset(t, 'a', 1 << 16);
    bad |= run("degenerate a x 65536", t, 1 << 16);
    for (uint64_t n = 2; n < (1u << 20); n = n * 7 + 3) {
        char nm[64];
        oracle_gen_text(t, n, n, dna, 4);
        snprintf(nm, sizeof nm, "dna");
        bad |= run(nm, t, n);
        oracle_gen_text(t, n, n + 1, all, 256);   /* 0x00 and 0xFF included */
        snprintf(nm, sizeof nm, "byte256");
        bad |= run(nm, t, n);
        oracle_gen_text(t, n, n + 2, bin, 2);
        snprintf(nm, sizeof nm, "binary");
        bad |= run(nm, t, n);
    }
    for (uint64_t i = 0; i < 4096; ++i) t[i] = "abaab"[i % 5];   /* periodic */
    bad |= run("periodic abaab", t, 4096);
    free(t);
    return bad;
}
