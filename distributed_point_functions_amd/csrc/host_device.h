// host_device.h — host-side HIP plumbing shared by the Tier-2 objects
// (csrc/dpf.cc, csrc/dcf.cc): status mapping, the per-thread stream and a
// stream-ordered device buffer.
#pragma once

#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "dpf_amd.h"
#include "dpf_amd/status.h"
#include "internal.h"

namespace distributed_point_functions {
namespace dpf_internal_host {


inline Status HipStatus(hipError_t e, const char* what) {
  if (e == hipSuccess) return OkStatus();
  if (e == hipErrorOutOfMemory)
    return ResourceExhaustedError(std::string(what) + ": " + hipGetErrorString(e));
  return InternalError(std::string(what) + ": " + hipGetErrorString(e));
}

inline Status AbiStatus(int rc) {
  if (rc == DPF_AMD_OK) return OkStatus();
  return Status(static_cast<StatusCode>(rc), dpf_amd::LastError());
}

// The calling thread's stream, destroyed when the thread exits (a server
// answering from many short-lived threads does not accumulate streams).
inline hipStream_t ThreadStream() {
  struct Holder {
    hipStream_t s = nullptr;
    Holder() {
      if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) s = nullptr;
    }
    ~Holder() {
      if (s) hipStreamDestroy(s);
    }
  };
  thread_local Holder h;
  return h.s;
}

// Host-side phase timer: with DPF_AMD_TRACE_HOST set, Mark(name) prints the
// wall time since the previous mark to stderr (the reference has no tracing;
// this is how the Tier-2 host overhead is attributed).
class HostTrace {
 public:
  explicit HostTrace(const char* scope)
      : scope_(scope), on_(std::getenv("DPF_AMD_TRACE_HOST") != nullptr),
        t_(std::chrono::steady_clock::now()) {}
  void Mark(const char* phase) {
    if (!on_) return;
    const auto now = std::chrono::steady_clock::now();
    std::fprintf(stderr, "[dpf_amd] %s/%s %.3f ms\n", scope_, phase,
                 std::chrono::duration<double, std::milli>(now - t_).count());
    t_ = now;
  }

 private:
  const char* scope_;
  bool on_;
  std::chrono::steady_clock::time_point t_;
};

// Host layouts with holes (e.g. {uint32_t, uint64_t}: 16 bytes, 4 unused):
// the kernels write only the scalars, so a buffer whose rows reach the caller
// is cleared first and stale device memory never shows up in the padding.
inline bool HasPadding(const dpf_amd_value_type& vt) {
  int used = 0;
  for (int i = 0; i < vt.num_scalars; ++i) used += vt.scalars[i].bytes;
  return used < vt.out_stride;
}

inline Status ClearPadding(const dpf_amd_value_type& vt, void* p, size_t bytes, hipStream_t s) {
  if (bytes == 0 || !HasPadding(vt)) return OkStatus();
  return HipStatus(hipMemsetAsync(p, 0, bytes, s), "hipMemsetAsync");
}

class DeviceBuffer {
 public:
  DeviceBuffer() = default;
  ~DeviceBuffer() { Reset(); }
  DeviceBuffer(const DeviceBuffer&) = delete;
  DeviceBuffer& operator=(const DeviceBuffer&) = delete;
  Status Alloc(size_t bytes, hipStream_t s) {
    Reset();
    stream_ = s;
    if (bytes == 0) bytes = 16;
    return HipStatus(hipMallocAsync(&p_, bytes, s), "hipMallocAsync");
  }
  Status Upload(const void* src, size_t bytes, hipStream_t s) {
    DPF_RETURN_IF_ERROR(Alloc(bytes, s));
    if (bytes == 0) return OkStatus();
    return HipStatus(hipMemcpyAsync(p_, src, bytes, hipMemcpyHostToDevice, s), "upload");
  }
  void Reset() {
    if (p_) (void)hipFreeAsync(p_, stream_);
    p_ = nullptr;
  }
  void* get() const { return p_; }
  template <typename T>
  T* as() const {
    return static_cast<T*>(p_);
  }

 private:
  void* p_ = nullptr;
  hipStream_t stream_ = nullptr;
};

}  // namespace dpf_internal_host
}  // namespace distributed_point_functions
