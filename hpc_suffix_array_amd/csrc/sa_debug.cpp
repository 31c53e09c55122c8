#include <execinfo.h>
#include <signal.h>
#include <unistd.h>
#include <cstdlib>
#include <cstdio>
static void on_segv(int sig) {
    void* fr[64];
    int k = backtrace(fr, 64);
    fprintf(stderr, "libsa_hip debug: signal %d, backtrace:\n", sig);
    backtrace_symbols_fd(fr, k, 2);
    _exit(128 + sig);
}
__attribute__((constructor)) static void sa_debug_init() {
    if (getenv("SA_DEBUG_SEGV")) signal(SIGSEGV, on_segv);
}
