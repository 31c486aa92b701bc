// host_write_probe.hip (round 5) — can the host write a call's small inputs
// (a key's seed and correction words, ~2.3 KiB) straight into device memory,
// so that the walk kernel needs no copy kernel in front of it?  On the
// per-call EvaluateAt path the copy kernel costs 2.3 us plus a 6 us
// dependent-dispatch gap (rocprofv3 trace of cpp_api_bench c2).  Allocates
// fine-grained device memory (hipExtMallocWithFlags, hipDeviceMallocFinegrained),
// reports whether the device is large-BAR and what hipPointerGetAttributes
// says, then (only with a host-visible pointer) 200 rounds of: host memcpy of
// a fresh 2,320-byte pattern, kernel launch that checks every word, sync —
// against the same rounds with a copy kernel from pinned memory.
// Not part of the library:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/experiments/host_write_probe.hip \
//     -o tools/experiments/host_write_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <vector>

#define CK(x)                                                                \
  do {                                                                       \
    hipError_t e = (x);                                                      \
    if (e != hipSuccess) {                                                   \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, \
                  __LINE__);                                                 \
      std::exit(1);                                                          \
    }                                                                        \
  } while (0)

constexpr int kWords = 580;  // 2,320 bytes

__global__ void KCheck(const uint32_t* p, uint32_t seed, uint32_t* bad) {
  for (int i = threadIdx.x; i < kWords; i += blockDim.x)
    if (p[i] != seed * 2654435761u + (uint32_t)i) atomicAdd(bad, 1u);
}
__global__ void KCopy(uint32_t* d, const uint32_t* s) {
  for (int i = threadIdx.x; i < kWords; i += blockDim.x) d[i] = s[i];
}

int main() {
  int dev = 0, large = 0;
  CK(hipDeviceGetAttribute(&large, hipDeviceAttributeIsLargeBar, dev));
  uint32_t* fg = nullptr;
  CK(hipExtMallocWithFlags((void**)&fg, 1 << 20, hipDeviceMallocFinegrained));
  hipPointerAttribute_t at;
  CK(hipPointerGetAttributes(&at, fg));
  std::printf("{\"large_bar\": %d, \"type\": %d, \"device_ptr\": \"%p\", \"host_ptr\": \"%p\"}\n",
              large, (int)at.type, at.devicePointer, at.hostPointer);
  uint32_t* bad;
  CK(hipMalloc(&bad, 4));
  CK(hipMemset(bad, 0, 4));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  uint32_t* pin;
  CK(hipHostMalloc((void**)&pin, kWords * 4, hipHostMallocMapped | hipHostMallocCoherent));
  uint32_t* pin_dev;
  CK(hipHostGetDevicePointer((void**)&pin_dev, pin, 0));
  uint32_t* dbuf;
  CK(hipMalloc(&dbuf, kWords * 4));
  std::vector<uint32_t> pat(kWords);
  const int rounds = 200;
  auto fill = [&](int r) {
    for (int i = 0; i < kWords; ++i) pat[i] = (uint32_t)r * 2654435761u + (uint32_t)i;
  };
  // copy-kernel path (the library's current upload of small parts)
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < rounds; ++r) {
    fill(r);
    std::memcpy(pin, pat.data(), kWords * 4);
    hipLaunchKernelGGL(KCopy, dim3(1), dim3(256), 0, s, dbuf, pin_dev);
    hipLaunchKernelGGL(KCheck, dim3(1), dim3(256), 0, s, dbuf, (uint32_t)r, bad);
    CK(hipStreamSynchronize(s));
  }
  auto t1 = std::chrono::steady_clock::now();
  uint32_t nbad = 0;
  CK(hipMemcpy(&nbad, bad, 4, hipMemcpyDeviceToHost));
  std::printf("{\"path\": \"copy_kernel\", \"us_per_round\": %.2f, \"bad_words\": %u}\n",
              std::chrono::duration<double, std::micro>(t1 - t0).count() / rounds, nbad);
  // host writes into fine-grained device memory
  uint32_t* hp = (uint32_t*)at.hostPointer;
  if (!hp && large) hp = fg;  // large BAR: the device address may be host-mapped
  if (!hp) {
    std::printf("{\"path\": \"host_write\", \"skipped\": \"no host pointer\"}\n");
    return 0;
  }
  CK(hipMemset(bad, 0, 4));
  t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < rounds; ++r) {
    fill(r);
    std::memcpy(hp, pat.data(), kWords * 4);
    std::atomic_thread_fence(std::memory_order_seq_cst);
    hipLaunchKernelGGL(KCheck, dim3(1), dim3(256), 0, s, fg, (uint32_t)r, bad);
    CK(hipStreamSynchronize(s));
  }
  t1 = std::chrono::steady_clock::now();
  CK(hipMemcpy(&nbad, bad, 4, hipMemcpyDeviceToHost));
  std::printf("{\"path\": \"host_write\", \"us_per_round\": %.2f, \"bad_words\": %u}\n",
              std::chrono::duration<double, std::micro>(t1 - t0).count() / rounds, nbad);
  // the check kernel alone (launch + sync floor)
  t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < rounds; ++r) {
    hipLaunchKernelGGL(KCheck, dim3(1), dim3(256), 0, s, dbuf, (uint32_t)(rounds - 1), bad);
    CK(hipStreamSynchronize(s));
  }
  t1 = std::chrono::steady_clock::now();
  std::printf("{\"path\": \"check_only\", \"us_per_round\": %.2f}\n",
              std::chrono::duration<double, std::micro>(t1 - t0).count() / rounds);
  return 0;
}
