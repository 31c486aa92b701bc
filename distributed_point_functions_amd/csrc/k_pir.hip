// k_pir.hip — dense-PIR XOR scan (pir/internal/inner_product_hwy.cc:157-258
// semantics), the partial / share XOR folds and the incremental-output gather.
#include <hip/hip_runtime.h>

#include "kernel_args.h"

namespace dpf_amd {

// ----------------------------------------------------------------------------
// Gather / fold helpers
// ----------------------------------------------------------------------------

__global__ void KGatherRows(int64_t n, const int64_t* src_offset, int64_t opp,
                            int64_t stride, const char* in, char* out) {
  const int64_t total = n * opp * stride;
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < total; b += step) {
    const int64_t row = b / stride, byte = b % stride;
    const int64_t i = row / opp, k = row % opp;
    out[b] = in[(src_offset[i] + k) * stride + byte];
  }
}

// XOR of num_parts equally sized partial vectors.  A 256-thread block owns
// kFoldWords consecutive 16-byte words; its threads split the parts into
// kFoldSlices interleaved slices (loads of one part stay contiguous), then the
// slices are folded through LDS.  Keeps many independent loads in flight, so
// a 2048-part fold of a few hundred bytes costs microseconds, not a serial
// chain of 2048 dependent loads.

__global__ __launch_bounds__(256) void KXorFold(const uint4* parts, int num_parts,
                                                int64_t words, uint4* out) {
  __shared__ uint4 red[kFoldSlices][kFoldWords];
  const int w = threadIdx.x % kFoldWords;
  const int s = threadIdx.x / kFoldWords;
  const int64_t i = (int64_t)blockIdx.x * kFoldWords + w;
  uint4 acc = make_uint4(0, 0, 0, 0);
  if (i < words) {
#pragma unroll 8
    for (int p = s; p < num_parts; p += kFoldSlices) {
      const uint4 v = parts[(int64_t)p * words + i];
      acc.x ^= v.x;
      acc.y ^= v.y;
      acc.z ^= v.z;
      acc.w ^= v.w;
    }
  }
  red[s][w] = acc;
  __syncthreads();
  for (int half = kFoldSlices / 2; half > 0; half >>= 1) {
    if (s < half) {
      const uint4 o = red[s + half][w];
      uint4 m = red[s][w];
      m.x ^= o.x;
      m.y ^= o.y;
      m.z ^= o.z;
      m.w ^= o.w;
      red[s][w] = m;
    }
    __syncthreads();
  }
  if (s == 0 && i < words) out[i] = red[0][w];
}

__global__ void KXorFoldBytes(const uint8_t* parts, int num_parts, int64_t bytes,
                              uint8_t* out) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < bytes; i += step) {
    uint8_t acc = 0;
    for (int p = 0; p < num_parts; ++p) acc ^= parts[(int64_t)p * bytes + i];
    out[i] = acc;
  }
}

// ----------------------------------------------------------------------------
// Dense PIR XOR scan (pir/internal/inner_product_hwy.cc:157-258 semantics)
// ----------------------------------------------------------------------------
//
// A wave owns tiles of 128 records (one selection block per query).  Within
// a record slice of Cs <= 64 16-byte chunks, lane l reads chunk l % Cs of
// record l / Cs (64 / Cs records per wave-instruction, fully coalesced
// 16-byte loads), and XORs it into per-query accumulators under the
// selection-bit mask.  Records wider than 1 KiB are split into 64-chunk
// slices over gridDim.y.  Partials (per block, query, chunk) are folded by
// KXorFold.

__device__ __forceinline__ uint32_t SelWord(const uint4& s, int idx) {
  return idx == 0 ? s.x : idx == 1 ? s.y : idx == 2 ? s.z : s.w;
}

template <int QN>
__global__ __launch_bounds__(kScanBlock) void KPirScan(ScanArgs a) {
  __shared__ uint4 red[kScanBlock];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int chunk_lo = blockIdx.y * 64;
  const int Cs = min(64, a.C - chunk_lo);
  const int G = 64 / Cs;
  const bool active = lane < G * Cs;
  const int my_chunk = chunk_lo + (lane % Cs);
  const int my_rec = lane / Cs;
  uint4 acc[QN];
#pragma unroll
  for (int q = 0; q < QN; ++q) acc[q] = make_uint4(0, 0, 0, 0);

  const int64_t tiles = (a.num_records + 127) >> 7;
  const int64_t wstride = (int64_t)gridDim.x * kScanWaves;
  for (int64_t tile = (int64_t)blockIdx.x * kScanWaves + wave; tile < tiles; tile += wstride) {
    uint4 sw[QN];
#pragma unroll
    for (int q = 0; q < QN; ++q)
      sw[q] = (q < a.nq) ? a.sel[(int64_t)(a.q0 + q) * a.sel_blocks + tile]
                         : make_uint4(0, 0, 0, 0);
    const int64_t rec0 = tile << 7;
    for (int it = 0; it < 128; it += G * kScanUnroll) {
      uint4 v[kScanUnroll];
      int rr[kScanUnroll];
#pragma unroll
      for (int u = 0; u < kScanUnroll; ++u) {
        rr[u] = it + u * G + my_rec;
        const int64_t rec = rec0 + rr[u];
        const bool ok = active && rr[u] < 128 && rec < a.num_records;
        v[u] = ok ? a.db[rec * a.C + my_chunk] : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < kScanUnroll; ++u) {
        const int r = rr[u] & 127;
#pragma unroll
        for (int q = 0; q < QN; ++q) {
          const uint32_t m = 0u - ((SelWord(sw[q], r >> 5) >> (r & 31)) & 1u);
          acc[q].x ^= v[u].x & m;
          acc[q].y ^= v[u].y & m;
          acc[q].z ^= v[u].z & m;
          acc[q].w ^= v[u].w & m;
        }
      }
    }
  }
  // Fold lanes that share a chunk, then waves, through LDS.
  for (int q = 0; q < a.nq && q < QN; ++q) {
    uint4 mine = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int qq = 0; qq < QN; ++qq)
      if (qq == q) mine = acc[qq];
    red[threadIdx.x] = active ? mine : make_uint4(0, 0, 0, 0);
    __syncthreads();
    if (threadIdx.x < Cs) {
      uint4 r = make_uint4(0, 0, 0, 0);
      for (int w = 0; w < kScanWaves; ++w)
        for (int g = 0; g < G; ++g) {
          uint4 x = red[w * 64 + g * Cs + threadIdx.x];
          r.x ^= x.x;
          r.y ^= x.y;
          r.z ^= x.z;
          r.w ^= x.w;
        }
      a.partials[((int64_t)blockIdx.x * a.total_q + a.q0 + q) * a.C + chunk_lo + threadIdx.x] = r;
    }
    __syncthreads();
  }
}

int LaunchGatherRows(int grid, hipStream_t st, int64_t n, const int64_t* src_offset,
                     int64_t opp, int64_t stride, const char* in, char* out) {
  hipLaunchKernelGGL(KGatherRows, dim3(grid), dim3(256), 0, st, n, src_offset, opp, stride,
                     in, out);
  return LaunchCheck("gather kernel launch");
}

int LaunchXorFold(unsigned blocks, hipStream_t st, const uint4* parts, int num_parts,
                  int64_t words, uint4* out) {
  hipLaunchKernelGGL(KXorFold, dim3(blocks), dim3(256), 0, st, parts, num_parts, words, out);
  return LaunchCheck("xor fold kernel launch");
}

int LaunchXorFoldBytes(int grid, hipStream_t st, const uint8_t* parts, int num_parts,
                       int64_t bytes, uint8_t* out) {
  hipLaunchKernelGGL(KXorFoldBytes, dim3(grid), dim3(256), 0, st, parts, num_parts, bytes,
                     out);
  return LaunchCheck("xor fold kernel launch");
}

int LaunchPirScan(int nq, dim3 g, hipStream_t st, const ScanArgs& a) {
  if (nq == 1)
    hipLaunchKernelGGL((KPirScan<1>), g, dim3(kScanBlock), 0, st, a);
  else if (nq <= 2)
    hipLaunchKernelGGL((KPirScan<2>), g, dim3(kScanBlock), 0, st, a);
  else if (nq <= 4)
    hipLaunchKernelGGL((KPirScan<4>), g, dim3(kScanBlock), 0, st, a);
  else
    hipLaunchKernelGGL((KPirScan<8>), g, dim3(kScanBlock), 0, st, a);
  return LaunchCheck("pir scan kernel launch");
}

}  // namespace dpf_amd
