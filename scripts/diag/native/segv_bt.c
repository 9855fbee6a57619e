// Diagnosis helper (CPU side only): on SIGSEGV print the native backtrace of the faulting thread
// to stderr, then re-raise with the default action.  Loaded with ctypes by tests/conftest.py when
// DTD_SEGV_BT=1, to locate a host-side crash inside a runtime library (symbols exported by the
// libraries show up; static functions show as offsets).
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static void on_segv(int sig, siginfo_t* si, void* ctx) {
  (void)ctx;
  void* frames[64];
  const char hdr[] = "\n[segv_bt] native backtrace:\n";
  write(2, hdr, sizeof(hdr) - 1);
  int n = backtrace(frames, 64);
  backtrace_symbols_fd(frames, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

__attribute__((visibility("default"))) int segv_bt_install(void) {
  struct sigaction sa;
  memset(&sa, 0, sizeof(sa));
  sa.sa_sigaction = on_segv;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  return sigaction(SIGSEGV, &sa, 0);
}
