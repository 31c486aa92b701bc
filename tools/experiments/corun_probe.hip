// corun_probe.hip (round 5) — can VALU-bound bitsliced AES waves run beside
// LDS-bound T-table AES waves on the same CUs and add throughput?  Times the
// T-table value-PRG pair hash (KTable) alone at 2 and 1 blocks per CU, the
// bitsliced one (KBitsliced) alone, and both at once on two streams (KTable
// held to 1 block per CU by dynamic LDS so the bitsliced blocks fit beside it).
// Built like bsaes_bench.hip (needs bsaes_gen.h from gen_bsaes.py).
// Derived from bsaes_bench.hip:
// the LDS T-table AES (HashWords<1, 2, true>, the fused kernel's current leaf
// hash) against the generated bitsliced AES (bsaes_gen.h, 16 pairs per lane).
// Checks that both produce identical words, then times each over a large
// grid.  Not part of the library: generate bsaes_gen.h first
// (python tools/experiments/gen_bsaes.py), then
//   hipcc --offload-arch=gfx950 -O3 -I distributed_point_functions_amd/csrc \
//     -I include tools/experiments/bsaes_bench.hip -o bsaes_bench
#include <hip/hip_runtime.h>

#include <chrono>
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
  const int tt = argc > 1 ? std::atoi(argv[1]) : (3 << 19);  // T-table threads
  const int bt = argc > 2 ? std::atoi(argv[2]) : (1 << 18);  // bitsliced threads
  const int reps = argc > 3 ? std::atoi(argv[3]) : 8;
  const int extra_lds = argc > 4 ? std::atoi(argv[4]) : 40 << 10;
  uint32_t *d1, *d2;
  CK(hipMalloc(&d1, (size_t)tt * 4));
  CK(hipMalloc(&d2, (size_t)bt * 4));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t a0, a1, b0, b1;
  CK(hipEventCreate(&a0));
  CK(hipEventCreate(&a1));
  CK(hipEventCreate(&b0));
  CK(hipEventCreate(&b1));
  const double tblocks = (double)tt * reps * 32, bblocks = (double)bt * reps * 32;
  auto run = [&](int mode, float* ta, float* tb, float* wall) {
    // mode 0: T-table (2/CU) alone, 1: T-table (1/CU) alone, 2: bitsliced
    // alone, 3: T-table (1/CU) + bitsliced together
    for (int w = 0; w < 2; ++w) {
      CK(hipDeviceSynchronize());
      const auto t0 = std::chrono::steady_clock::now();
      if (mode != 2) {
        CK(hipEventRecord(a0, s1));
        hipLaunchKernelGGL(KTable, dim3(tt / 768), dim3(768), mode == 0 ? 0 : extra_lds, s1, d1, 0,
                           reps);
        CK(hipEventRecord(a1, s1));
      }
      if (mode >= 2) {
        CK(hipEventRecord(b0, s2));
        hipLaunchKernelGGL(KBitsliced, dim3(bt / 256), dim3(256), 0, s2, d2, 0, reps);
        CK(hipEventRecord(b1, s2));
      }
      CK(hipDeviceSynchronize());
      *wall = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    *ta = *tb = 0;
    if (mode != 2) CK(hipEventElapsedTime(ta, a0, a1));
    if (mode >= 2) CK(hipEventElapsedTime(tb, b0, b1));
  };
  for (int rep = 0; rep < 2; ++rep) {
    float ta, tb, wall;
    run(0, &ta, &tb, &wall);
    std::printf("T-table 2/CU alone:  %.3f ms, %.1f G blocks/s\n", ta, tblocks / (ta * 1e-3) / 1e9);
    run(1, &ta, &tb, &wall);
    std::printf("T-table 1/CU alone:  %.3f ms, %.1f G blocks/s\n", ta, tblocks / (ta * 1e-3) / 1e9);
    run(2, &ta, &tb, &wall);
    std::printf("bitsliced alone:     %.3f ms, %.1f G blocks/s\n", tb, bblocks / (tb * 1e-3) / 1e9);
    run(3, &ta, &tb, &wall);
    std::printf("together: T-table %.3f ms, bitsliced %.3f ms, wall %.3f ms: %.1f G blocks/s "
                "combined\n", ta, tb, wall, (tblocks + bblocks) / (wall * 1e-3) / 1e9);
  }
  return 0;
}
