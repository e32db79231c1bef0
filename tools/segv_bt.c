/* Diagnostic helper (tools only, never linked into the product): on SIGSEGV print the native backtrace. */
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

static void on_segv(int sig) {
    void* frames[64];
    int n = backtrace(frames, 64);
    backtrace_symbols_fd(frames, n, 2);
    _exit(128 + sig);
}

void segv_bt_install(void) { signal(SIGSEGV, on_segv); }
