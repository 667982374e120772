// Native crash report (SURVEY.md §5 failure detection): on SIGSEGV / SIGBUS / SIGFPE / SIGILL /
// SIGABRT in any thread, print the faulting address and the native call stack (module +
// offset per frame; `addr2line -f -C -e <module> <offset>` against the shipped .so names the
// function and line), then hand the signal to the handler that was installed before -- Python's
// faulthandler (PYTHONFAULTHANDLER=1 / pytest) prints every thread's Python stack next.
// Installed once, the first time an engine is created (engine.cpp ccfd_engine_create), or on
// request (ccfd_crash_report_install).  Async-signal-safe: write(2) + backtrace(3) only (the
// backtrace buffer is static; glibc's unwinder is loaded at install time, not in the handler).
#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <unistd.h>

#include <atomic>
#include <cstdint>
#include <cstring>

namespace {

constexpr int kSigs[] = {SIGSEGV, SIGBUS, SIGFPE, SIGILL, SIGABRT};
constexpr int kNSigs = sizeof(kSigs) / sizeof(kSigs[0]);
struct sigaction g_prev[kNSigs];
std::atomic<int> g_installed{0};
void* g_frames[64];

void put(const char* s) {
  ssize_t r = write(2, s, std::strlen(s));
  (void)r;
}

void put_hex(uintptr_t v) {
  char b[19] = "0x";
  for (int i = 0; i < 16; ++i) {
    const int d = (int)((v >> (60 - 4 * i)) & 0xf);
    b[2 + i] = (char)(d < 10 ? '0' + d : 'a' + d - 10);
  }
  b[18] = 0;
  put(b);
}

void handler(int sig, siginfo_t* si, void* uc) {
  put("\n[ccfd] native crash: signal ");
  char n[4] = {(char)('0' + sig / 10), (char)('0' + sig % 10), 0, 0};
  put(n);
  put(" at address ");
  put_hex(reinterpret_cast<uintptr_t>(si ? si->si_addr : nullptr));
  put("\n[ccfd] native stack (module+offset):\n");
  const int k = backtrace(g_frames, 64);
  for (int i = 0; i < k; ++i) {
    Dl_info info;
    put("  #");
    char idx[4] = {(char)('0' + i / 10), (char)('0' + i % 10), ' ', 0};
    put(idx);
    if (dladdr(g_frames[i], &info) && info.dli_fname) {
      put(info.dli_fname);
      put("+");
      put_hex(reinterpret_cast<uintptr_t>(g_frames[i]) - reinterpret_cast<uintptr_t>(info.dli_fbase));
      if (info.dli_sname) {
        put(" (");
        put(info.dli_sname);
        put(")");
      }
    } else {
      put_hex(reinterpret_cast<uintptr_t>(g_frames[i]));
    }
    put("\n");
  }
  // chain: the previous handler (faulthandler) or the default action
  for (int i = 0; i < kNSigs; ++i) {
    if (kSigs[i] != sig) continue;
    const struct sigaction& p = g_prev[i];
    if (p.sa_flags & SA_SIGINFO) {
      if (p.sa_sigaction) { p.sa_sigaction(sig, si, uc); return; }
    } else if (p.sa_handler != SIG_IGN && p.sa_handler != SIG_DFL && p.sa_handler) {
      p.sa_handler(sig);
      return;
    }
    signal(sig, SIG_DFL);
    raise(sig);
    return;
  }
}

}  // namespace

// Returns how many signals it (re)installed: a runtime loaded later (HSA / HIP, torch) may
// have put its own handler in front; calling again puts this one back in front of it.
extern "C" int ccfd_crash_report_install() {
  static std::atomic<int> busy{0};
  int expect = 0;
  if (!busy.compare_exchange_strong(expect, 1)) return 0;
  if (!g_installed.exchange(1)) backtrace(g_frames, 2);   // load the unwinder now, not in the handler
  int n = 0;
  for (int i = 0; i < kNSigs; ++i) {
    struct sigaction cur;
    if (sigaction(kSigs[i], nullptr, &cur) == 0 && (cur.sa_flags & SA_SIGINFO) && cur.sa_sigaction == handler)
      continue;                            // already in front
    struct sigaction sa;
    std::memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = handler;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    sigaction(kSigs[i], &sa, &g_prev[i]);
    ++n;
  }
  busy.store(0);
  return n;
}
