// host_common.cc — error state and buffer management of the C ABI.
#include <execinfo.h>
#include <signal.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

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
// the previous handler.
struct sigaction g_prev[32];
void OnFatal(int sig, siginfo_t* info, void* uctx) {
  char msg[128];
  const int n = snprintf(msg, sizeof msg, "[dpf_amd] signal %d at address %p, thread stack:\n",
                         sig, info ? info->si_addr : nullptr);
  if (n > 0) (void)!write(2, msg, static_cast<size_t>(n));
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
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_sigaction = OnFatal;
  sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
  sigemptyset(&sa.sa_mask);
  for (int sig : {SIGSEGV, SIGBUS, SIGABRT}) sigaction(sig, &sa, &g_prev[sig]);
  return true;
}();
}  // namespace

}  // namespace dpf_amd

extern "C" {

const char* dpf_amd_last_error(void) { return dpf_amd::LastError(); }

void dpf_amd_free(void* p) { free(p); }

}  // extern "C"
