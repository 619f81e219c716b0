/* Test-harness aid: on SIGSEGV print the native backtrace (the frames of
 * libcfd_hip.so and the HIP runtime that Python's faulthandler cannot show),
 * then hand the signal to the handler installed before (faulthandler's).
 * Loaded by tests/conftest.py on the GPU box only; never part of the product. */
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

static struct sigaction prev_sa;

static void on_segv(int sig, siginfo_t* si, void* uc) {
    (void)uc;
    char msg[96];
    int n = snprintf(msg, sizeof msg, "\nnative backtrace (SIGSEGV at %p):\n", si ? si->si_addr : 0);
    if (n > 0) (void)!write(2, msg, (size_t)n);
    void* buf[64];
    const int k = backtrace(buf, 64);
    backtrace_symbols_fd(buf, k, 2);
    sigaction(SIGSEGV, &prev_sa, NULL);
    raise(sig);
}

int segv_bt_install(void) {
    void* warm[2];
    backtrace(warm, 2); /* load the unwinder now, not inside the handler */
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = on_segv;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    return sigaction(SIGSEGV, &sa, &prev_sa);
}
