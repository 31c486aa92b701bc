// dispatch_spread_probe.hip (round 5) — how long does the dispatcher take to
// start one launch's workgroups?  One key's 16,384-point EvaluateAt
// (KEvaluatePointsQuad<1, true>: 256 blocks x 256 threads, 128 KiB of LDS
// tables per block) showed its blocks starting over 3.95 us of an 83.5 us
// span (tools/quad_trace.py).  Each block of this probe stamps
// s_memrealtime (100 MHz) at entry; the spread (last - first entry) is
// printed per shape: 256 blocks of 64 / 256 / 1024 threads with 0, 64 or 128
// KiB of static LDS, and 512 / 1024 blocks of 256 threads with no LDS.
// Not part of the library:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/experiments/dispatch_spread_probe.hip \
//     -o tools/experiments/dispatch_spread_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
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

template <int LDS_WORDS>
__global__ __launch_bounds__(1024) void KSpread(uint64_t* stamp, uint32_t* sink) {
  if (threadIdx.x == 0) stamp[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
  if constexpr (LDS_WORDS > 0) {
    __shared__ uint32_t tab[LDS_WORDS];
    tab[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (tab[(threadIdx.x * 7) & 255] == 0xffffffffu) sink[0] = 1;
  }
}

// the quad walk's shape: a 1.7 KiB argument block, ~96 VGPRs, 128 KiB LDS
struct BigArgs {
  uint32_t w[432];
};
__global__ __launch_bounds__(256) __attribute__((amdgpu_num_vgpr(96))) void KSpreadBig(
    uint64_t* stamp, uint32_t* sink, BigArgs b) {
  if (threadIdx.x == 0) stamp[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
  __shared__ uint32_t tab[32768];
  tab[threadIdx.x] = threadIdx.x ^ b.w[threadIdx.x & 255];
  __syncthreads();
  if (tab[(threadIdx.x * 7) & 255] == 0xffffffffu) sink[0] = b.w[431];
}

static void RunBig() {
  const int blocks = 256;
  uint64_t* d;
  uint32_t* sink;
  CK(hipMalloc(&d, sizeof(uint64_t) * blocks));
  CK(hipMalloc(&sink, 4));
  BigArgs b{};
  std::vector<uint64_t> h(blocks);
  std::vector<double> spreads;
  for (int rep = 0; rep < 7; ++rep) {
    hipLaunchKernelGGL(KSpreadBig, dim3(blocks), dim3(256), 0, 0, d, sink, b);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h.data(), d, sizeof(uint64_t) * blocks, hipMemcpyDeviceToHost));
    const auto mm = std::minmax_element(h.begin(), h.end());
    if (rep > 0) spreads.push_back((*mm.second - *mm.first) / 100.0);
  }
  std::sort(spreads.begin(), spreads.end());
  std::printf("{\"shape\": \"big_args_96_vgprs_lds_128k\", \"blocks\": 256, \"threads\": 256, "
              "\"start_spread_us_median\": %.2f, \"min\": %.2f, \"max\": %.2f}\n",
              spreads[spreads.size() / 2], spreads.front(), spreads.back());
  CK(hipFree(d));
  CK(hipFree(sink));
}

template <int LDS_WORDS>
static void Run(const char* name, int blocks, int threads) {
  uint64_t* d;
  uint32_t* sink;
  CK(hipMalloc(&d, sizeof(uint64_t) * blocks));
  CK(hipMalloc(&sink, 4));
  std::vector<uint64_t> h(blocks);
  std::vector<double> spreads;
  for (int rep = 0; rep < 7; ++rep) {
    hipLaunchKernelGGL(KSpread<LDS_WORDS>, dim3(blocks), dim3(threads), 0, 0, d, sink);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h.data(), d, sizeof(uint64_t) * blocks, hipMemcpyDeviceToHost));
    const auto mm = std::minmax_element(h.begin(), h.end());
    if (rep > 0) spreads.push_back((*mm.second - *mm.first) / 100.0);
  }
  std::sort(spreads.begin(), spreads.end());
  std::printf("{\"shape\": \"%s\", \"blocks\": %d, \"threads\": %d, \"lds_kib\": %d, "
              "\"start_spread_us_median\": %.2f, \"min\": %.2f, \"max\": %.2f}\n",
              name, blocks, threads, LDS_WORDS * 4 / 1024, spreads[spreads.size() / 2],
              spreads.front(), spreads.back());
  CK(hipFree(d));
  CK(hipFree(sink));
}

int main() {
  Run<0>("no_lds", 256, 256);
  Run<16384>("lds_64k", 256, 256);
  Run<32768>("lds_128k_quad_walk_shape", 256, 256);
  Run<32768>("lds_128k_64_threads", 256, 64);
  Run<32768>("lds_128k_1024_threads", 256, 1024);
  Run<0>("no_lds_512_blocks", 512, 256);
  Run<0>("no_lds_1024_blocks", 1024, 256);
  Run<0>("no_lds_64_threads", 256, 64);
  RunBig();
  return 0;
}
