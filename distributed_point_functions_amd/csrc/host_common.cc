// host_common.cc — error state and buffer management of the C ABI.
#include <stdlib.h>

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

}  // namespace dpf_amd

extern "C" {

const char* dpf_amd_last_error(void) { return dpf_amd::LastError(); }

void dpf_amd_free(void* p) { free(p); }

}  // extern "C"
