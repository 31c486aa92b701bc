// host_common.cc — error state and buffer management of the C ABI.
#include <execinfo.h>
#include <signal.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <atomic>
#include <string>

#include "dpf_amd.h"
#include "internal.h"

namespace dpf_amd {

namespace {
thread_local std::string g_last_error;
}

int SetError(int code, const std::string& message) {
  g_last_error = message;
  return code;
}

const char* LastError() { return g_last_error.c_str(); }

namespace {
// DPF_AMD_SEGV_BACKTRACE=1 (diagnostics): on SIGSEGV / SIGBUS / SIGABRT
// print the faulting thread's native stack to stderr (a host process's
// Python faulthandler shows only Python frames), then hand the signal to
// the previous handler.  The handler only calls async-signal-safe code:
// write(2) of a message built by hand, and backtrace(), whose first call
// (which loads libgcc_s and allocates) already happened when the handler
// was installed.
struct sigaction g_prev[32];
size_t AppendStr(char* buf, size_t at, size_t cap, const char* s) {
  while (*s && at + 1 < cap) buf[at++] = *s++;
  return at;
}
size_t AppendHex(char* buf, size_t at, size_t cap, uintptr_t v) {
  char tmp[2 + 2 * sizeof(uintptr_t)];
  int k = 0;
  do {
    tmp[k++] = "0123456789abcdef"[v & 15];
    v >>= 4;
  } while (v && k < static_cast<int>(sizeof tmp));
  at = AppendStr(buf, at, cap, "0x");
  while (k > 0 && at + 1 < cap) buf[at++] = tmp[--k];
  return at;
}
void OnFatal(int sig, siginfo_t* info, void* uctx) {
  char msg[128];
  size_t n = AppendStr(msg, 0, sizeof msg, "[dpf_amd] signal ");
  if (n + 3 < sizeof msg) {
    if (sig >= 10) msg[n++] = static_cast<char>('0' + (sig / 10) % 10);
    msg[n++] = static_cast<char>('0' + sig % 10);
  }
  n = AppendStr(msg, n, sizeof msg, " at address ");
  n = AppendHex(msg, n, sizeof msg, reinterpret_cast<uintptr_t>(info ? info->si_addr : nullptr));
  n = AppendStr(msg, n, sizeof msg, ", thread stack:\n");
  (void)!write(2, msg, n);
  void* frames[64];
  const int k = backtrace(frames, 64);
  backtrace_symbols_fd(frames, k, 2);
  struct sigaction& prev = g_prev[sig];
  if (prev.sa_flags & SA_SIGINFO) {
    if (prev.sa_sigaction) prev.sa_sigaction(sig, info, uctx);
  } else if (prev.sa_handler != SIG_IGN && prev.sa_handler != SIG_DFL) {
    prev.sa_handler(sig);
  } else {
    signal(sig, SIG_DFL);
    raise(sig);
  }
}
const bool g_segv_trace = [] {
  if (!getenv("DPF_AMD_SEGV_BACKTRACE")) return false;
  void* warm[4];
  (void)backtrace(warm, 4);  // loads libgcc_s now, not inside the handler
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = OnFatal;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigemptyset(&sa.sa_mask);
  for (int sig : {SIGSEGV, SIGBUS, SIGABRT}) sigaction(sig, &sa, &g_prev[sig]);
  return true;
}();

// Idle per-thread resource objects kept for future threads (ThreadRecycled,
// host_device.h); DPF_AMD_THREAD_CACHE or dpf_amd_set_thread_cache_cap.
std::atomic<int> g_thread_cache_cap{[] {
  const char* e = getenv("DPF_AMD_THREAD_CACHE");
  return e ? atoi(e) : 64;
}()};
std::atomic<int> g_force_peer_copies{0};
thread_local int t_prefix_expand = 0;  // 0 automatic, 1 off, 2 host bookkeeping
}  // namespace

int ThreadCacheCap() { return g_thread_cache_cap.load(std::memory_order_relaxed); }
bool ForcePeerCopies() { return g_force_peer_copies.load(std::memory_order_relaxed) != 0; }
bool PrefixExpandOff() {
  static const bool env_off = [] {
    const char* e = getenv("DPF_AMD_PREFIX_EXPAND");
    return e && atoi(e) == 0;
  }();
  return env_off || t_prefix_expand == 1;
}
bool HostIncremental() {
  static const bool env_host = [] {
    const char* e = getenv("DPF_AMD_HOST_INCREMENTAL");
    return e && atoi(e) != 0;
  }();
  return env_host || t_prefix_expand == 2;
}

}  // namespace dpf_amd

extern "C" {

const char* dpf_amd_last_error(void) { return dpf_amd::LastError(); }

void dpf_amd_free(void* p) { free(p); }

int dpf_amd_set_thread_cache_cap(int cap) {
  if (cap < 0) return dpf_amd::SetError(DPF_AMD_INVALID_ARGUMENT, "cap must be >= 0");
  dpf_amd::g_thread_cache_cap.store(cap);
  return DPF_AMD_OK;
}

void dpf_amd_set_force_peer_copies(int on) { dpf_amd::g_force_peer_copies.store(on ? 1 : 0); }

int dpf_amd_set_prefix_expand(int mode) {
  if (mode < 0 || mode > 2) return -2;
  const int prev = dpf_amd::t_prefix_expand;
  dpf_amd::t_prefix_expand = mode;
  return prev;
}

}  // extern "C"
