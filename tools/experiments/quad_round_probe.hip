// quad_round_probe.hip (round 5) — where do the ~160 cycles of a quad-lane
// AES round go?  The latency-bound launches (one key's 16,384-point
// EvaluateAt, KEvaluatePointsQuad; c1's KExpandCoop walk) run one wave per
// SIMD through a dependent chain of quad rounds (aes_device.h AesQuadRk).
// This probe times chains of N rounds in isolation with s_memtime (shader
// clock) and s_memrealtime (100 MHz), per mode:
//   0  AesQuadRk<true>  (four tables, the production round of the EvaluateAt walk)
//   1  AesQuadRk<false> (two tables + rotl16)
//   2  pure LDS chain: v_perm -> one ds_read_b32 -> xor, per step
//   3  four lookups of the lane's own column, xor3 combine, no DPP
//      (perm -> 4 ds_read -> xor3: the round without its cross-lane moves)
//   4  mode 2 with one active lane
//   5  AesQuad<true> (two tables, per-round masked key XOR: KExpandCoop's walk)
// at 1, 4 and 8 waves per CU (one block per CU: 128 KiB of tables).
// Not part of the library:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I distributed_point_functions_amd/csrc \
//     -I include tools/experiments/quad_round_probe.hip -o tools/experiments/quad_round_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "aes_device.h"

using namespace dpf_amd;

#define CK(x)                                                                \
  do {                                                                       \
    hipError_t e = (x);                                                      \
    if (e != hipSuccess) {                                                   \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, \
                  __LINE__);                                                 \
      std::exit(1);                                                          \
    }                                                                        \
  } while (0)

template <int MODE>
__global__ __launch_bounds__(512) void KQuadProbe(uint32_t* out, unsigned long long* cyc,
                                                  int iters) {
  __shared__ uint32_t tab[kTab4Words];
  FillTables4(tab);
  __syncthreads();
  const Lds4 L = MakeLds4(tab);
  const int c = threadIdx.x & 3;
  const QuadRk k = MakeQuadRk<0>(c);
  const QuadKey kl = MakeQuadKey<0>(c);
  const QuadDiff kd = MakeQuadDiff(c);
  const uint32_t m = 0u - ((threadIdx.x >> 2) & 1u);
  uint32_t w = (threadIdx.x * 0x9e3779b9u) ^ (blockIdx.x * 0x85ebca6bu);
  if (MODE == 4 && (threadIdx.x & 63) != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll 1
  for (int i = 0; i < iters; ++i) {
    if constexpr (MODE == 0) {
      w = AesQuadRk<true>(w, k, L);
    } else if constexpr (MODE == 1) {
      w = AesQuadRk<false>(w, k, LdsOf(L));
    } else if constexpr (MODE == 5) {
      w = AesQuad<true>(w, kl, kd, m, LdsOf(L));
    } else if constexpr (MODE == 2 || MODE == 4) {
#pragma unroll
      for (int r = 0; r < 10; ++r) w ^= LoadT0(LdsOf(L), w, r & 3);
    } else {
#pragma unroll
      for (int r = 0; r < 10; ++r) {
        const uint32_t u0 = LoadT0(LdsOf(L), w, 0), u1 = LoadT1(LdsOf(L), w, 1),
                       u2 = LoadT2(L, w, 2), u3 = LoadT3(L, w, 3);
        w = Xor3(u0, u1, Xor3(u2, u3, k.rk[r]));
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = w;
  if ((threadIdx.x & 63) == 0) {
    const int wv = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    cyc[2 * wv] = t1 - t0;
    cyc[2 * wv + 1] = r1 - r0;
  }
}

template <int MODE>
static void Run(const char* name, int threads, int iters) {
  const int blocks = 256;
  uint32_t* out;
  unsigned long long* cyc;
  const int waves = blocks * threads / 64;
  CK(hipMalloc(&out, sizeof(uint32_t) * blocks * threads));
  CK(hipMalloc(&cyc, sizeof(unsigned long long) * 2 * waves));
  CK(hipMemset(cyc, 0, sizeof(unsigned long long) * 2 * waves));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  std::vector<unsigned long long> h(2 * waves);
  for (int rep = 0; rep < 5; ++rep) {
    CK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(KQuadProbe<MODE>, dim3(blocks), dim3(threads), 0, 0, out, cyc, iters);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  CK(hipMemcpy(h.data(), cyc, sizeof(unsigned long long) * 2 * waves, hipMemcpyDeviceToHost));
  double sc = 0, sr = 0;
  int n = 0;
  for (int i = 0; i < waves; ++i)
    if (h[2 * i]) {
      sc += (double)h[2 * i];
      sr += (double)h[2 * i + 1];
      ++n;
    }
  sc /= n;
  sr /= n;
  const double rounds = 10.0 * iters;
  std::printf(
      "{\"mode\": \"%s\", \"waves_per_cu\": %d, \"rounds\": %.0f, \"memtime_cycles_per_round\": %.1f, "
      "\"ns_per_round\": %.2f, \"memtime_mhz\": %.0f, \"event_ms\": %.4f}\n",
      name, threads / 64, rounds, sc / rounds, sr * 10.0 / rounds, sc / sr * 100.0, best);
  CK(hipFree(out));
  CK(hipFree(cyc));
}

int main() {
  const int iters = 2000;  // 20,000 rounds per chain
  for (int threads : {64, 256, 512}) {
    Run<0>("quad_t4", threads, iters);
    Run<1>("quad_t2", threads, iters);
    Run<2>("lds_chain", threads, iters);
    Run<3>("own_column_4_lookups", threads, iters);
    Run<4>("lds_chain_one_lane", threads, iters);
    Run<5>("quad_masked_t2", threads, iters);
  }
  return 0;
}
