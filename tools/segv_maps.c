// segv_maps.c — diagnostic only (never loaded by the product): on SIGSEGV / SIGBUS, write the
// faulting address, the raw backtrace with dladdr() names and /proc/self/maps to stderr, then
// hand the signal to the previously installed handler (rocprofv3's glog handler, Python's
// faulthandler). Loaded by bench.py when RLP_SEGV_DIAG=1 (ctypes), to symbolise the frames of a
// crash inside the profiler-wrapped HIP runtime (profiles/r4/r4i_pmc_crash.txt).
// Build: gcc -O1 -g -shared -fPIC tools/segv_maps.c -o tools/segv_maps.so -ldl
#define _GNU_SOURCE
#include <dlfcn.h>
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

static struct sigaction old_segv, old_bus;
static char altstack[1 << 16];

static void put(const char *s) { (void)!write(2, s, strlen(s)); }

static void handler(int sig, siginfo_t *si, void *uc) {
    char buf[512];
    snprintf(buf, sizeof buf, "\n=== segv_maps: signal %d at address %p ===\n", sig, si->si_addr);
    put(buf);
    void *fr[64];
    const int n = backtrace(fr, 64);
    for (int i = 0; i < n; ++i) {
        Dl_info di;
        if (dladdr(fr[i], &di) && di.dli_fname) {
            snprintf(buf, sizeof buf, "  #%02d %p %s+0x%lx (%s+0x%lx)\n", i, fr[i], di.dli_fname,
                     (unsigned long)((char *)fr[i] - (char *)di.dli_fbase),
                     di.dli_sname ? di.dli_sname : "?",
                     di.dli_saddr ? (unsigned long)((char *)fr[i] - (char *)di.dli_saddr) : 0ul);
        } else {
            snprintf(buf, sizeof buf, "  #%02d %p ?\n", i, fr[i]);
        }
        put(buf);
    }
    put("=== /proc/self/maps ===\n");
    const int fd = open("/proc/self/maps", O_RDONLY);
    if (fd >= 0) {
        ssize_t k;
        while ((k = read(fd, buf, sizeof buf)) > 0) (void)!write(2, buf, (size_t)k);
        close(fd);
    }
    put("=== end segv_maps ===\n");
    // restore the previous handler and return: the faulting access repeats and reaches it
    sigaction(SIGSEGV, &old_segv, NULL);
    sigaction(SIGBUS, &old_bus, NULL);
    (void)uc;
}

__attribute__((constructor)) static void install(void) {
    stack_t ss;
    ss.ss_sp = altstack;
    ss.ss_size = sizeof altstack;
    ss.ss_flags = 0;
    sigaltstack(&ss, NULL);
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = handler;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    sigaction(SIGSEGV, &sa, &old_segv);
    sigaction(SIGBUS, &sa, &old_bus);
}
