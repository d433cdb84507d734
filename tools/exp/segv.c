// SIGSEGV handler printing a native backtrace (loaded with ctypes before a
// reproduction run; host-side debugging aid).
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

static void handler(int sig, siginfo_t* si, void* ctx)
{
    (void)ctx;
    void* bt[64];
    char msg[128];
    int n = snprintf(msg, sizeof(msg), "\n*** signal %d at address %p, backtrace:\n", sig, si->si_addr);
    write(2, msg, n);
    int k = backtrace(bt, 64);
    backtrace_symbols_fd(bt, k, 2);
    _exit(139);
}

__attribute__((constructor)) static void install(void)
{
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = handler;
    sa.sa_flags = SA_SIGINFO;
    sigaction(SIGSEGV, &sa, NULL);
}
