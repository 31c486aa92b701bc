// bsaes_bench.hip — standalone A/B of the value-PRG pair hash on gfx950:
// the LDS T-table AES (HashWords<1, 2, true>, the fused kernel's current leaf
// hash) against the generated bitsliced AES (bsaes_gen.h, 16 pairs per lane).
// Checks that both produce identical words, then times each over a large
// grid.  Not part of the library: generate bsaes_gen.h first
// (python tools/experiments/gen_bsaes.py), then
//   hipcc --offload-arch=gfx950 -O3 -I distributed_point_functions_amd/csrc \
//     -I include tools/experiments/bsaes_bench.hip -o bsaes_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "aes_device.h"
#include "bsaes_gen.h"

using namespace dpf_amd;

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, \
                  __LINE__);                                               \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

__device__ __forceinline__ uint32_t Mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// Seed i of thread t (bit 0 clear, as after control-bit extraction).
__device__ __forceinline__ void SeedOf(uint32_t t, int i, uint32_t (&s)[4]) {
  const uint32_t b = t * 16u + (uint32_t)i;
  s[0] = Mix(b * 4u + 0u) & ~1u;
  s[1] = Mix(b * 4u + 1u);
  s[2] = Mix(b * 4u + 2u);
  s[3] = Mix(b * 4u + 3u);
}

// out[t][i] = {h0 words 0..3, h1 word 0} when `full`, else an XOR digest.
__global__ __launch_bounds__(768) void KTable(uint32_t* out, int full, int reps) {
  __shared__ uint32_t tab[kTabWords];
  FillTables(tab);
  __syncthreads();
  const Lds L = MakeLds(tab);
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (int r = 0; r < reps; ++r) {
    for (int i = 0; i < 16; ++i) {
      uint32_t x[1][4];
      SeedOf(t + (uint32_t)r * 0x9e3779b9u, i, x[0]);
      uint32_t h[1][2][4];
      HashWords<1, 2, true>(x, h, L);
      if (full) {
        uint32_t* o = out + ((size_t)t * 16 + i) * 5;
        for (int c = 0; c < 4; ++c) o[c] = h[0][0][c];
        o[4] = h[0][1][0];
      }
      acc ^= h[0][0][0] ^ h[0][0][1] ^ h[0][0][2] ^ h[0][0][3] ^ h[0][1][0];
    }
  }
  if (!full) out[t] = acc;
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
void KBitsliced(uint32_t* out, int full, int reps) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (int r = 0; r < reps; ++r) {
    uint32_t sg[16][4];
    for (int i = 0; i < 16; ++i) {
      uint32_t s[4];
      SeedOf(t + (uint32_t)r * 0x9e3779b9u, i, s);
      Sigma(s, sg[i]);
    }
    uint32_t h0[16][4], h1[16];
    BsAesPairs16(sg, h0, h1);
    // sigma words again (the fused kernel reloads them instead); the asm
    // keeps the compiler from reusing the first computation across the AES
    uint32_t tt = t + (uint32_t)r * 0x9e3779b9u;
    asm volatile("" : "+v"(tt));
    for (int i = 0; i < 16; ++i) {
      uint32_t s[4], g[4];
      SeedOf(tt, i, s);
      Sigma(s, g);
      for (int c = 0; c < 4; ++c) h0[i][c] = Xor3(h0[i][c], g[c], kBsK10[c]);
      h1[i] = Xor3(h1[i], g[0], kBsK10[0]);
    }
    for (int i = 0; i < 16; ++i) {
      if (full) {
        uint32_t* o = out + ((size_t)t * 16 + i) * 5;
        for (int c = 0; c < 4; ++c) o[c] = h0[i][c];
        o[4] = h1[i];
      }
      acc ^= h0[i][0] ^ h0[i][1] ^ h0[i][2] ^ h0[i][3] ^ h1[i];
    }
  }
  if (!full) out[t] = acc;
}

int main(int argc, char** argv) {
  const int check_threads = 3 << 14;  // multiple of 768 and 256
  const int grid_threads = argc > 1 ? std::atoi(argv[1]) : (3 << 20);
  const int reps = argc > 2 ? std::atoi(argv[2]) : 4;
  uint32_t *a, *b;
  CK(hipMalloc(&a, (size_t)check_threads * 16 * 5 * 4));
  CK(hipMalloc(&b, (size_t)check_threads * 16 * 5 * 4));
  hipLaunchKernelGGL(KTable, dim3(check_threads / 768), dim3(768), 0, 0, a, 1, 1);
  hipLaunchKernelGGL(KBitsliced, dim3(check_threads / 256), dim3(256), 0, 0, b, 1, 1);
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> ha((size_t)check_threads * 80), hb((size_t)check_threads * 80);
  CK(hipMemcpy(ha.data(), a, ha.size() * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hb.data(), b, hb.size() * 4, hipMemcpyDeviceToHost));
  size_t bad = 0;
  for (size_t i = 0; i < ha.size(); ++i) bad += ha[i] != hb[i];
  std::printf("check: %zu of %zu words differ (T-table vs bitsliced)\n", bad, ha.size());
  if (bad && !(argc > 3 && argv[3][0] == 'x')) {
    for (int i = 0; i < 10; ++i) std::printf("  %08x %08x\n", ha[i], hb[i]);
    return 1;
  }
  CK(hipFree(a));
  CK(hipFree(b));
  uint32_t* d;
  CK(hipMalloc(&d, (size_t)grid_threads * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int k = 0; k < 2; ++k) {
    for (int w = 0; w < 2; ++w) {  // warm-up + timed
      CK(hipEventRecord(e0));
      if (k == 0)
        hipLaunchKernelGGL(KTable, dim3(grid_threads / 768), dim3(768), 0, 0, d, 0, reps);
      else
        hipLaunchKernelGGL(KBitsliced, dim3(grid_threads / 256), dim3(256), 0, 0, d, 0, reps);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
    }
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double blocks = (double)grid_threads * reps * 32;
    std::printf("%s: %.3f ms, %.1f G AES blocks/s\n", k == 0 ? "T-table  " : "bitsliced",
                ms, blocks / (ms * 1e-3) / 1e9);
  }
  return 0;
}
