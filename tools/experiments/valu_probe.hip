// valu_probe.hip — issue-rate probe of v_bitop3_b32 on gfx950 (measurement
// tool, not part of the library): 3-VGPR-operand bitop3 with operands in
// distinct / identical VGPR banks (v mod 4), with an inline-constant third
// operand, and a dependent chain, at 1..8 waves per SIMD.
#include <hip/hip_runtime.h>

#include <cstdio>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      std::printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                            \
    }                                                                      \
  } while (0)

// 16 independent bitop3 per iteration; destinations v40..v55, sources chosen
// per variant.  Registers are clobbered explicitly.
#define CLOB                                                                   \
  "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", \
      "v51", "v52", "v53", "v54", "v55", "v1", "v2", "v3", "v4", "v5", "v6",    \
      "v8", "v12", "v16", "v20"

template <int V>
__global__ void KProbe(unsigned* out, int iters) {
  unsigned x = threadIdx.x;
  asm volatile(
      "v_mov_b32 v1, %0\n v_mov_b32 v2, %0\n v_mov_b32 v3, %0\n v_mov_b32 v4, %0\n"
      "v_mov_b32 v5, %0\n v_mov_b32 v6, %0\n v_mov_b32 v8, %0\n v_mov_b32 v12, %0\n"
      "v_mov_b32 v16, %0\n v_mov_b32 v20, %0\n" ::"v"(x)
      : CLOB);
  for (int i = 0; i < iters; ++i) {
    if constexpr (V == 0) {  // distinct banks: v1 (b1), v2 (b2), v3 (b3) -> dst bank 0..3
      asm volatile(
#define L(d) "v_bitop3_b32 v" #d ", v1, v2, v3 bitop3:0x96\n"
          L(40) L(41) L(42) L(43) L(44) L(45) L(46) L(47) L(48) L(49) L(50) L(51) L(52)
              L(53) L(54) L(55)
#undef L
          ::: CLOB);
    } else if constexpr (V == 1) {  // same bank: v4, v8, v12 (bank 0)
      asm volatile(
#define L(d) "v_bitop3_b32 v" #d ", v4, v8, v12 bitop3:0x96\n"
          L(40) L(41) L(42) L(43) L(44) L(45) L(46) L(47) L(48) L(49) L(50) L(51) L(52)
              L(53) L(54) L(55)
#undef L
          ::: CLOB);
    } else if constexpr (V == 2) {  // two VGPRs (distinct banks) + inline constant
      asm volatile(
#define L(d) "v_bitop3_b32 v" #d ", v1, v2, 0 bitop3:0x96\n"
          L(40) L(41) L(42) L(43) L(44) L(45) L(46) L(47) L(48) L(49) L(50) L(51) L(52)
              L(53) L(54) L(55)
#undef L
          ::: CLOB);
    } else if constexpr (V == 3) {  // two VGPRs same bank + constant
      asm volatile(
#define L(d) "v_bitop3_b32 v" #d ", v4, v8, 0 bitop3:0x96\n"
          L(40) L(41) L(42) L(43) L(44) L(45) L(46) L(47) L(48) L(49) L(50) L(51) L(52)
              L(53) L(54) L(55)
#undef L
          ::: CLOB);
    } else if constexpr (V == 4) {  // dependent chain through v40
      asm volatile(
#define L(d) "v_bitop3_b32 v40, v40, v2, v3 bitop3:0x96\n"
          L(40) L(41) L(42) L(43) L(44) L(45) L(46) L(47) L(48) L(49) L(50) L(51) L(52)
              L(53) L(54) L(55)
#undef L
          ::: CLOB);
    } else {  // 4 interleaved dependent chains, distinct banks
      asm volatile(
          "v_bitop3_b32 v40, v40, v2, v3 bitop3:0x96\n"
          "v_bitop3_b32 v41, v41, v2, v3 bitop3:0x96\n"
          "v_bitop3_b32 v42, v42, v1, v3 bitop3:0x96\n"
          "v_bitop3_b32 v43, v43, v1, v2 bitop3:0x96\n"
          "v_bitop3_b32 v40, v40, v2, v3 bitop3:0x96\n"
          "v_bitop3_b32 v41, v41, v2, v3 bitop3:0x96\n"
          "v_bitop3_b32 v42, v42, v1, v3 bitop3:0x96\n"
          "v_bitop3_b32 v43, v43, v1, v2 bitop3:0x96\n"
          "v_bitop3_b32 v40, v40, v2, v3 bitop3:0x96\n"
          "v_bitop3_b32 v41, v41, v2, v3 bitop3:0x96\n"
          "v_bitop3_b32 v42, v42, v1, v3 bitop3:0x96\n"
          "v_bitop3_b32 v43, v43, v1, v2 bitop3:0x96\n"
          "v_bitop3_b32 v40, v40, v2, v3 bitop3:0x96\n"
          "v_bitop3_b32 v41, v41, v2, v3 bitop3:0x96\n"
          "v_bitop3_b32 v42, v42, v1, v3 bitop3:0x96\n"
          "v_bitop3_b32 v43, v43, v1, v2 bitop3:0x96\n" ::
              : CLOB);
    }
  }
  unsigned r;
  asm volatile("v_mov_b32 %0, v40" : "=v"(r)::CLOB);
  if (r == 0x12345u) out[0] = r;
}

template <int V>
int Run(const char* name, unsigned* d) {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  const int iters = 4096;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int waves = 1; waves <= 8; waves *= 2) {
    // one workgroup per CU of 4 * waves wave64s = `waves` waves per SIMD
    const int block = 256 * waves > 1024 ? 1024 : 256 * waves;
    const int grid = cus * (256 * waves / block);
    float ms = 0;
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(KProbe<V>, dim3(grid), dim3(block), 0, 0, d, iters);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
    }
    const double instr = (double)grid * block / 64 * iters * 16;  // wave-instructions
    // cycles per wave-instruction per SIMD at the measured time, 2.4 GHz nominal
    const double per_simd = instr / (cus * 4.0);
    std::printf("%-28s waves/SIMD %d: %.3f ms, %.2f cyc/instr/SIMD @2.4GHz\n", name, waves, ms,
                ms * 1e-3 * 2.4e9 / per_simd);
  }
  return 0;
}

int main() {
  unsigned* d;
  CK(hipMalloc(&d, 64));
  Run<0>("3 VGPR, distinct banks", d);
  Run<1>("3 VGPR, same bank", d);
  Run<2>("2 VGPR + const", d);
  Run<3>("2 VGPR same bank + const", d);
  Run<4>("dependent chain", d);
  Run<5>("4 dependent chains", d);
  return 0;
}
