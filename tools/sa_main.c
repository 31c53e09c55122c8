/*
 * tools/sa_main.c -- command-line driver with the stdout contract of the
 * reference's src/sequential/main_sequential.c:52-162, running the GPU
 * builder of libsa_hip.so.  Built as bin/main_sequential (and linked as
 * bin/cuda_suffix_array, the binary scripts/benchmark_cuda_kaggle.py:108 of
 * the reference expects), so the reference's harness parses it unchanged:
 *   "Actual string length: N", "Longest repeated substring: '...' (length:
 *   N)", "Total execution time: X", ===STRUCTURED_RESULTS=== TOTAL_TIME /
 *   SA_TIME / LCP_TIME (main_sequential.c:38-50,122-154), plus "Kernel time:"
 *   and "GPU memory used:" (benchmark_cuda_kaggle.py:32-49,95-102).
 * Timing follows the reference: SA_TIME = create + build (:97-109),
 * LCP_TIME = LCP + LRS (:112-117); validation is not timed (:120).
 * Differences: direct-string mode works (the reference segfaults there,
 * SURVEY.md 3A), and the file is read as raw bytes without NUL truncation
 * of the length.
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>

#include "../include/sa_hip.h"
#include "../include/suffix_array.h"

static double now_s(void) {
    struct timeval tv;
    gettimeofday(&tv, NULL);
    return tv.tv_sec + tv.tv_usec * 1e-6;
}

static char* read_all(const char* path, long* n) {
    FILE* f = fopen(path, "rb");
    if (!f) {
        fprintf(stderr, "Error: Cannot open file %s\n", path);
        return NULL;
    }
    fseek(f, 0, SEEK_END);
    *n = ftell(f);
    fseek(f, 0, SEEK_SET);
    if (*n <= 0) {
        fprintf(stderr, "Error: File is empty or cannot determine size\n");
        fclose(f);
        return NULL;
    }
    char* buf = (char*)malloc((size_t)*n + 1);
    if (!buf || fread(buf, 1, (size_t)*n, f) != (size_t)*n) {
        fprintf(stderr, "Error: failed to read %s\n", path);
        free(buf);
        fclose(f);
        return NULL;
    }
    buf[*n] = '\0';
    fclose(f);
    printf("Successfully read file: %s (%ld bytes)\n", path, *n);
    return buf;
}

static void print_span(const char* label, const char* s, long from, long count) {
    printf("%s %ld characters: \"", label, count);
    for (long i = from; i < from + count; i++) putchar(s[i] ? s[i] : ' ');
    printf("\"\n");
}

int main(int argc, char** argv) {
    if (argc != 2) {
        printf("Usage: %s <input_file_or_string>\n", argv[0]);
        printf("If argument contains '/' or '.', it's treated as a file\n");
        printf("Otherwise, it's treated as a direct string\n");
        return 1;
    }
    const char* impl = strstr(argv[0], "cuda") ? "hip_gpu" : "sequential";
    char* input;
    long n;
    const char* filename = argv[1];
    if (strchr(argv[1], '/') || strchr(argv[1], '.')) {
        printf("Reading from file: %s\n", argv[1]);
        input = read_all(argv[1], &n);
        if (!input) return 1;
        printf("File read successfully: %s\n", argv[1]);
        printf("Actual string length: %ld\n", n);
        if (n < 100) {
            printf("Full content: \"%s\"\n", input);
        } else {
            print_span("First", input, 0, 50);
            print_span("Last", input, n - 50, 50);
        }
        printf("\n");
    } else {
        input = strdup(argv[1]);
        n = (long)strlen(input);
        filename = "direct_string";
        printf("Input string: %s\n", input);
        printf("String length: %ld\n", n);
    }
    if (n > 0x7FFFFFFFL) {
        fprintf(stderr, "Error: the SuffixArray ABI holds int n (max 2^31-1); use sa_build_ex\n");
        return 1;
    }
    if (sa_device_count() <= 0) {
        fprintf(stderr, "Error: no HIP device visible (libsa_hip builds on an MI355X)\n");
        return 1;
    }

    double t0 = now_s();
    SuffixArray* sa = create_suffix_array(input, (int)n);
    if (!sa) {
        printf("Error: Failed to create suffix array\n");
        free(input);
        return 1;
    }
    sa_stats st;
    memset(&st, 0, sizeof st);
    if (sa_build_ex((const uint8_t*)sa->str, (uint64_t)n, sa->sa, 4, NULL, &st) != SA_OK) {
        fprintf(stderr, "Error: build failed: %s\n", sa_last_error());
        return 1;
    }
    double t_mid = now_s();
    build_lcp_array(sa);
    char* lrs = find_longest_repeated_substring(sa);
    double t_end = now_s();
    int valid = is_valid_suffix_array(sa);

    printf("\n=== RESULTS ===\n");
    printf("Valid suffix array: %s\n", valid ? "YES" : "NO");
    if (lrs)
        printf("Longest repeated substring: '%s' (length: %zu)\n", lrs, strlen(lrs));
    else
        printf("No repeated substring found\n");
    printf("Suffix array construction time: %.6f seconds\n", t_mid - t0);
    printf("LCP construction + LRS search time: %.6f seconds\n", t_end - t_mid);
    printf("Total execution time: %.6f seconds\n", t_end - t0);
    printf("Kernel time: %.3f ms (%d doubling rounds, H2D %.3f ms, D2H %.3f ms)\n", st.total_ms, st.rounds,
           st.h2d_ms, st.d2h_ms);
    printf("GPU memory used: %.1f MB\n", (double)sa_workspace_bytes((uint64_t)n) / (1024.0 * 1024.0));
    if (n <= 100) {
        printf("\n=== DETAILED ANALYSIS ===\n");
        printf("Suffix Array: [");
        for (int i = 0; i < sa->n && i < 20; i++) printf("%d%s", sa->sa[i], (i < sa->n - 1 && i < 19) ? ", " : "");
        printf("%s]\n", sa->n > 20 ? ", ..." : "");
        printf("\nLCP Array: [");
        for (int i = 0; i < sa->n && i < 20; i++) printf("%d%s", sa->lcp[i], (i < sa->n - 1 && i < 19) ? ", " : "");
        printf("%s]\n", sa->n > 20 ? ", ..." : "");
    }
    printf("\n===STRUCTURED_RESULTS===\n");
    printf("IMPLEMENTATION:%s\n", impl);
    printf("FILENAME:%s\n", filename);
    printf("FILE_SIZE:%ld\n", n);
    printf("TOTAL_TIME:%.6f\n", t_end - t0);
    printf("SA_TIME:%.6f\n", t_mid - t0);
    printf("LCP_TIME:%.6f\n", t_end - t_mid);
    printf("PROCESSES:%d\n", 1);
    printf("===END_RESULTS===\n\n");
    free(lrs);
    destroy_suffix_array(sa);
    free(input);
    return 0;
}
