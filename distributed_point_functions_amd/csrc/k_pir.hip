// k_pir.hip — dense-PIR XOR scan (pir/internal/inner_product_hwy.cc:157-258
// semantics), the partial / share XOR folds and the incremental-output gather.
#include <hip/hip_runtime.h>

#include "kernel_args.h"

namespace dpf_amd {

// DB records are read exactly once per scan pass, so they are issued as
// nontemporal loads (DPF_AMD_SCAN_NT=1, default): measured on MI355X at
// 2^26 x 256 B, Q = 1 2.75 -> 2.47 ms (6.25 -> 6.94 TB/s), Q = 8 2.96 -> 2.55,
// Q = 64 18.8 -> 15.5 ms.  DPF_AMD_SCAN_NT=0 restores plain loads for A/B.
#ifndef DPF_AMD_SCAN_NT
#define DPF_AMD_SCAN_NT 1
#endif
__device__ __forceinline__ uint4 LoadRecordWord(const uint4* p) {
#if DPF_AMD_SCAN_NT
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
#else
  return *p;
#endif
}

// ----------------------------------------------------------------------------
// Gather / fold helpers
// ----------------------------------------------------------------------------

// Source rows outside [0, in_rows - opp] are not read: the segment is
// skipped and *err set (callers that know the source size pass it; the C ABI
// entry passes INT64_MAX and no flag).
__device__ __forceinline__ bool GatherRowOk(int64_t r, int64_t opp, int64_t in_rows, int* err) {
  if (r >= 0 && r <= in_rows - opp) return true;
  if (err) *err = 1;
  return false;
}

__global__ void KGatherRows(int64_t n, const int64_t* src_offset, int64_t opp,
                            int64_t stride, const char* in, char* out, int64_t in_rows,
                            int* err) {
  const int64_t total = n * opp * stride;
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; b < total; b += step) {
    const int64_t row = b / stride, byte = b % stride;
    const int64_t i = row / opp, k = row % opp;
    const int64_t r = src_offset[i];
    if (GatherRowOk(r, opp, in_rows, err)) out[b] = in[(r + k) * stride + byte];
  }
}

// 16-byte variant: every segment (opp x stride bytes) is a whole number of
// 16-byte words at a 16-byte-aligned source offset.
__global__ void KGatherRows16(int64_t n, const int64_t* src_offset, int64_t seg_words,
                              int64_t src_words_per_unit, const uint4* in, uint4* out,
                              int64_t opp, int64_t in_rows, int* err) {
  const int64_t total = n * seg_words;
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < total; w += step) {
    const int64_t i = w / seg_words, k = w - i * seg_words;
    const int64_t r = src_offset[i];
    if (GatherRowOk(r, opp, in_rows, err)) out[w] = in[r * src_words_per_unit + k];
  }
}

// As KGatherRows16 for strides that divide 16 (1, 2, 4, 8-byte rows):
// source row r starts word r / rows_per_word when r is a multiple of
// rows_per_word (EvaluateUntil's offsets are multiples of opp); other
// segments are copied byte-wise.
__global__ void KGatherRowsSmall(int64_t n, const int64_t* src_offset, int64_t seg_words,
                                 int64_t rows_per_word, const uint4* in, uint4* out,
                                 int64_t opp, int64_t in_rows, int* err) {
  const int64_t total = n * seg_words;
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; w < total; w += step) {
    const int64_t i = w / seg_words, k = w - i * seg_words;
    const int64_t r = src_offset[i];
    if (!GatherRowOk(r, opp, in_rows, err)) continue;
    if (r % rows_per_word == 0) {
      out[w] = in[r / rows_per_word + k];
    } else {
      const uint8_t* src = reinterpret_cast<const uint8_t*>(in) + r * (16 / rows_per_word) + 16 * k;
      uint8_t* dst = reinterpret_cast<uint8_t*>(out + w);
      for (int b = 0; b < 16; ++b) dst[b] = src[b];
    }
  }
}

// Host-to-device upload as a kernel on the caller's stream: 16-byte words
// (the tail byte-wise) read from pinned host memory mapped into the device
// address space.
__global__ void KCopyFromHost(char* dst, const char* src, int64_t bytes) {
  const int64_t words = bytes / 16;
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  const int64_t first = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int64_t w = first; w < words; w += step)
    reinterpret_cast<uint4*>(dst)[w] = reinterpret_cast<const uint4*>(src)[w];
  for (int64_t b = words * 16 + first; b < bytes; b += step) dst[b] = src[b];
}

int CopyFromMappedHost(void* dst, const void* mapped_src, size_t bytes, void* stream) {
  if (bytes == 0) return DPF_AMD_OK;
  if ((uintptr_t)dst % 16 || (uintptr_t)mapped_src % 16)
    return SetError(DPF_AMD_INTERNAL, "upload buffers must be 16-byte aligned");
  const int64_t words = (int64_t)(bytes + 15) / 16;
  const int grid = (int)std::min<int64_t>(1024, (words + 255) / 256);
  hipLaunchKernelGGL(KCopyFromHost, dim3(grid), dim3(256), 0, (hipStream_t)stream, (char*)dst,
                     (const char*)mapped_src, (int64_t)bytes);
  return LaunchCheck("upload kernel launch");
}

// XOR of num_parts equally sized partial vectors.  A 256-thread block owns
// kFoldWords consecutive 16-byte words; its threads split the parts into
// kFoldSlices interleaved slices (loads of one part stay contiguous), then the
// slices are folded through LDS.  Keeps many independent loads in flight, so
// a 2048-part fold of a few hundred bytes costs microseconds, not a serial
// chain of 2048 dependent loads.

// `clear` (the parts, or nullptr): every word is written back as zero after
// its one read, so atomic fold slots are left zeroed for the next scan.
__global__ __launch_bounds__(256) void KXorFold(const uint4* parts, int num_parts,
                                                int64_t words, uint4* out, uint4* clear) {
  __shared__ uint4 red[kFoldSlices][kFoldWords];
  const int w = threadIdx.x % kFoldWords;
  const int s = threadIdx.x / kFoldWords;
  const int64_t i = (int64_t)blockIdx.x * kFoldWords + w;
  uint4 acc = make_uint4(0, 0, 0, 0);
  if (i < words) {
#pragma unroll 8
    for (int p = s; p < num_parts; p += kFoldSlices) {
      const uint4 v = parts[(int64_t)p * words + i];
      if (clear) clear[(int64_t)p * words + i] = make_uint4(0, 0, 0, 0);
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

// Folds the per-lane accumulators of a block into partials
// [block][query][chunk]: lanes that share a chunk, then the block's waves,
// through LDS.
template <int QN>
__device__ __forceinline__ void FoldPartials(const ScanArgs& a, const uint4 (&acc)[QN],
                                             uint4* red, int Cs, int G, bool active,
                                             int chunk_lo, int64_t block) {
  for (int q = 0; q < a.nq && q < QN; ++q) {
    uint4 mine = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int qq = 0; qq < QN; ++qq)
      if (qq == q) mine = acc[qq];
    red[threadIdx.x] = active ? mine : make_uint4(0, 0, 0, 0);
    __syncthreads();
    if (threadIdx.x < Cs) {
      uint4 r = make_uint4(0, 0, 0, 0);
      // rolled: an unrolled G = 64 fold alone needs 256 VGPRs
#pragma unroll 1
      for (int w = 0; w < kScanWaves; ++w)
#pragma unroll 4
        for (int g = 0; g < G; ++g) {
          uint4 x = red[w * 64 + g * Cs + threadIdx.x];
          r.x ^= x.x;
          r.y ^= x.y;
          r.z ^= x.z;
          r.w ^= x.w;
        }
      const int64_t part = a.slots ? block % a.slots : block;
      uint4* dst = &a.partials[(part * a.total_q + a.q0 + q) * a.C + chunk_lo + threadIdx.x];
      if (a.slots) {
        // vector global atomics (per-lane addresses); XOR is order-free, so
        // the folded result is the same bytes whatever order blocks finish in
        unsigned int* d = reinterpret_cast<unsigned int*>(dst);
        atomicXor(d + 0, r.x);
        atomicXor(d + 1, r.y);
        atomicXor(d + 2, r.z);
        atomicXor(d + 3, r.w);
      } else {
        *dst = r;
      }
    }
    __syncthreads();
  }
}

// Masked XOR scan for any record width.  G records share a wave-instruction
// (G a power of two): G = 1 for C > 32 chunks (64-chunk slices of a record
// over gridDim.y, the last slice narrower), else the largest G with G * C <= 64
// (whole records, Cs = C chunks each).  Lanes past G * Cs repeat a load of
// their group and are dropped by FoldPartials.  For G <= 32 the records of one
// wave-instruction never straddle a 32-record selection word, so each query's
// word is wave-uniform (SGPRs) and a lane's mask is one signed bit-field
// extract; G = 64 (16-byte records) picks the lane's word of a uniform pair.
// The mask is applied with one v_bitop3 per dword; up to 16 queries per pass.
// G = 1 (records wider than 32 chunks): loads in flight per lane, and the
// slice-major grid — the slices of one tile range in consecutive logical
// blocks (a 1-D grid, slice = logical block % slices) instead of over
// gridDim.y, with consecutive logical blocks on one XCD (blocks are dealt
// round-robin over the 8 XCDs, each with its own L2): the slices of a tile
// range run together and share their boundary cache lines in one L2.
// Measured (profiles/ab_scan_g1_r06i/, alternated): 2^20 x 2 KiB Q = 1
// 0.461 -> 0.413 ms, 16 KiB 3.06 -> 2.93 ms, FETCH 19.19 -> 18.92 GB;
// slice-major without the XCD mapping 0.448 / 3.01; 16 loads in flight
// per lane the same within noise.
#ifndef DPF_SCAN_G1_U
#define DPF_SCAN_G1_U 8
#endif
#ifndef DPF_SCAN_G1_SLICE_MAJOR
#define DPF_SCAN_G1_SLICE_MAJOR 1
#endif
#ifndef DPF_SCAN_G1_XCD
#define DPF_SCAN_G1_XCD 1
#endif
// Four-Russians kernels over records wider than one 256-byte slice: the same
// slice-major, XCD-local block order.  With the wide-row grid sizing
// (kernels_capi.cc ScanGrid), alternated (profiles/ab_scan_wide_r06k/):
// 2^20 x 2 KiB Q = 10 / 100 0.64 / 1.12 -> 0.53 / 1.00 ms, 16 KiB 3.98 /
// 7.72 -> 3.70 / 6.07 ms (FETCH of the Q = 100 scan 31.7 -> 23.5 GB, its
// fold 6.7 -> 0.8 GB); c4 unchanged.
#ifndef DPF_SCAN_M4_SLICE_MAJOR
#define DPF_SCAN_M4_SLICE_MAJOR 1
#endif
// (part block, slice) of this block: a 1-D grid of blocks x slices when the
// launch is slice-major (ScanArgs::slice_major), else (blockIdx.x, blockIdx.y).
__device__ __forceinline__ void M4BlockSlice(const ScanArgs& a, int64_t& pb, int& slice) {
  if (!a.slice_major) {
    pb = blockIdx.x;
    slice = blockIdx.y;
    return;
  }
  const int slices = (a.C + 15) / 16;
  int64_t lb = blockIdx.x;
  const int64_t full = gridDim.x & ~7u;
  if (lb < full) lb = (lb & 7) * (full >> 3) + (lb >> 3);
  pb = lb / slices;
  slice = (int)(lb % slices);
}

// Progress-ordered wave priority for the grid-stride scans (A/B:
// DPF_SCAN_PRIO=1): a wave at iteration `it` of its `n` tiles runs at
// priority 3 - (quarter of its tiles done), so the sequencer's preference for
// older waves does not leave the last round's waves to finish one after
// another (KExpand's ProgressPrio, expand_device.h).  Wave-uniform.
#ifndef DPF_SCAN_PRIO
#define DPF_SCAN_PRIO 0  // KPirScanG and KPirScanM4Pair (A/B)
#endif
#ifndef DPF_SCAN_M4_PRIO
#define DPF_SCAN_M4_PRIO 1  // KPirScanM4 (c4 Q = 32 / 64 2.80 / 3.88 -> 2.73 / 3.78 ms)
#endif
template <bool ON = DPF_SCAN_PRIO != 0>
__device__ __forceinline__ void ScanPrio(int64_t it, int64_t n) {
  if constexpr (ON) {
    if (n < 4) return;
    if (it == 0) {
      __builtin_amdgcn_s_setprio(3);
      return;
    }
    const int64_t q = it * 4 / n;
    if (q == (it - 1) * 4 / n) return;
    if (q == 1)
      __builtin_amdgcn_s_setprio(2);
    else if (q == 2)
      __builtin_amdgcn_s_setprio(1);
    else
      __builtin_amdgcn_s_setprio(0);
  }
}

template <int QN, int G>
__global__ __launch_bounds__(kScanBlock) void KPirScanG(ScanArgs a) {
  constexpr int U = (G >= 64) ? 2 : (G == 1) ? DPF_SCAN_G1_U : (G * 8 <= 32) ? 8 : 32 / G;
  __shared__ uint4 red[kScanBlock];
  const int lane = threadIdx.x & 63;
  // wave-uniform by construction; readfirstlane lets the compiler see it, so
  // the selection words below are scalar loads into SGPRs
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr bool kSliceMajor = G == 1 && DPF_SCAN_G1_SLICE_MAJOR;
  const int slices = (a.C + 63) / 64;
  int64_t lb = blockIdx.x;  // logical block (slice-major grids)
  if (kSliceMajor && DPF_SCAN_G1_XCD) {
    const int64_t full = gridDim.x & ~7u;
    if (lb < full) lb = (lb & 7) * (full >> 3) + (lb >> 3);
  }
  const int64_t bx = kSliceMajor ? lb / slices : (int64_t)blockIdx.x;
  const int64_t gx = kSliceMajor ? (int64_t)(gridDim.x / slices) : (int64_t)gridDim.x;
  const int chunk_lo = (kSliceMajor ? (int)(lb % slices) : (int)blockIdx.y) * 64;
  const int Cs = (G == 1) ? min(64, a.C - chunk_lo) : a.C;
  const bool active = lane < G * Cs;
  const int my_chunk = chunk_lo + lane % Cs;
  const int my_rec = min(lane / Cs, G - 1);
  const uint32_t* sel = reinterpret_cast<const uint32_t*>(a.sel);
  uint4 acc[QN];
#pragma unroll
  for (int q = 0; q < QN; ++q) acc[q] = make_uint4(0, 0, 0, 0);
  const int64_t tiles = (a.num_records + 127) >> 7;
  const int64_t wstride = gx * kScanWaves;
  const int64_t tile0 = bx * kScanWaves + wave;
  const int64_t n_it = tile0 < tiles ? (tiles - tile0 + wstride - 1) / wstride : 0;
  for (int64_t tile = tile0; tile < tiles; tile += wstride) {
    ScanPrio((tile - tile0) / wstride, n_it);
    const int64_t rec0 = tile << 7;
    const bool full = rec0 + 128 <= a.num_records;
    if constexpr (G == 64) {
      // 128 records = 2 wave-instructions; lane l of half h is record
      // rec0 + 64h + l, selection bit l & 31 of word 2h + (l >> 5).
      uint4 v[U];
#pragma unroll
      for (int h = 0; h < U; ++h) {
        const int64_t rec = rec0 + 64 * h + lane;
        v[h] = (full || rec < a.num_records) ? LoadRecordWord(&a.db[rec])
                                              : make_uint4(0, 0, 0, 0);
      }
      const bool upper = lane >= 32;
#pragma unroll
      for (int q = 0; q < QN; ++q) {
        uint32_t w[4] = {0u, 0u, 0u, 0u};
        if (q < a.nq) {
#pragma unroll
          for (int d = 0; d < 4; ++d) w[d] = sel[((int64_t)(a.q0 + q) * a.sel_blocks + tile) * 4 + d];
        }
#pragma unroll
        for (int h = 0; h < U; ++h) {
          const uint32_t word = upper ? w[2 * h + 1] : w[2 * h];
          const uint32_t m = (uint32_t)__builtin_amdgcn_sbfe((int)word, lane & 31, 1);
          acc[q].x = __builtin_amdgcn_bitop3_b32(acc[q].x, v[h].x, m, 0x78);
          acc[q].y = __builtin_amdgcn_bitop3_b32(acc[q].y, v[h].y, m, 0x78);
          acc[q].z = __builtin_amdgcn_bitop3_b32(acc[q].z, v[h].z, m, 0x78);
          acc[q].w = __builtin_amdgcn_bitop3_b32(acc[q].w, v[h].w, m, 0x78);
        }
      }
    } else {
#pragma unroll 1
      for (int d = 0; d < 4; ++d) {
        // selection word d (records rec0 + 32d ..) of each query; with the
        // opt-in skip (ScanArgs::skip) their union masks the loads, so a
        // record no query of the pass selects is never fetched
        uint32_t word[QN];
        uint32_t need = a.skip ? 0u : ~0u;
#pragma unroll
        for (int q = 0; q < QN; ++q) {
          word[q] = (q < a.nq) ? sel[((int64_t)(a.q0 + q) * a.sel_blocks + tile) * 4 + d] : 0u;
          need |= word[q];
        }
#pragma unroll 1
        for (int k0 = 0; k0 < 32; k0 += G * U) {
          uint4 v[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int bit = k0 + u * G + my_rec;
            const int64_t rec = rec0 + d * 32 + bit;
            v[u] = ((full || rec < a.num_records) && ((need >> bit) & 1u))
                       ? LoadRecordWord(&a.db[rec * a.C + my_chunk])
                       : make_uint4(0, 0, 0, 0);
          }
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int bit = k0 + u * G + my_rec;
#pragma unroll
            for (int q = 0; q < QN; ++q) {
              const uint32_t m = (uint32_t)__builtin_amdgcn_sbfe((int)word[q], bit, 1);
              // acc ^= v & m as one v_bitop3 (truth table src0 ^ (src1 & src2))
              acc[q].x = __builtin_amdgcn_bitop3_b32(acc[q].x, v[u].x, m, 0x78);
              acc[q].y = __builtin_amdgcn_bitop3_b32(acc[q].y, v[u].y, m, 0x78);
              acc[q].z = __builtin_amdgcn_bitop3_b32(acc[q].z, v[u].z, m, 0x78);
              acc[q].w = __builtin_amdgcn_bitop3_b32(acc[q].w, v[u].w, m, 0x78);
            }
          }
        }
      }
    }
  }
  FoldPartials<QN>(a, acc, red, Cs, G, active, chunk_lo, bx);
}

// ----------------------------------------------------------------------------
// Many-query scan: method of Four Russians over 4-record groups
// ----------------------------------------------------------------------------
//
// The masked scan spends one VALU op per (query, record dword); at Q = 64 that
// is VALU-issue bound far above the HBM floor.  Here a wave reads a 256-byte
// column slice of 4 consecutive records (lane j = dword j, one coalesced
// load per record), builds the 16 XOR combinations of the 4 slices once in
// LDS (11 XORs, 15 row stores), and every query then costs ONE table row
// read — the row its 4 selection bits index — and the XORs of that row into
// its accumulators.  Lanes are (query, column part): 64 / P queries per wave,
// each lane owning 256 / P bytes of the slice as P-th of the row, read with
// ds_read_b128.  Table rows are 272 B apart, so the 16-byte slot of row e,
// column c is (e + c) mod 16: lanes of a ds_read_b128 group that read
// different rows hit different slots and lanes reading the same row
// broadcast — conflict-free for any selection.  Each wave owns its table (no
// block barrier); its accumulators are one partial of the fold
// (part = blockIdx.x * kScanM4Waves + wave, parts < a.parts).
//
// LDS traffic per 4 records: 15 row stores (64 lanes x 4 B) + QW rows read
// (256 B each); VALU: 11 + 2 + 64 XORs per lane.  Records past num_records
// and slice dwords past the record read as zero, so they add nothing.
//
// Measured on MI355X, c4 (2^26 x 256 B), Q = 64 (masked scan: 15.0 ms; two
// tables per step with XOR3 accumulators, ScanM4Tile2 below: 4.12 ms):
// this kernel 4.50 ms with ds_write_addtid row stores, 4.79 ms with
// ds_write2_b32 stores (7 address VGPRs).  Rejected: deeper register
// prefetch (2 / 4 groups at 2 waves/SIMD: 5.29 / 5.54 ms), row reads in
// batches of 4 (4.90), and tables shared by a block's waves (16 queries per
// wave, one LDS barrier per group, 8 waves/SIMD: 6.97 ms; Q = 100 in one
// pass 15.6 ms vs 9.2 in two per-wave passes).
#ifndef DPF_SCAN_M4_ADDTID
#define DPF_SCAN_M4_ADDTID 1  // row stores as ds_write_addtid_b32 (inline asm)
#endif
#ifndef DPF_SCAN_M4_WORD_LOOPS
#define DPF_SCAN_M4_WORD_LOOPS 1  // P = 2 / 4: per-word loops unrolled by two
#endif
#ifndef DPF_SCAN_M4_PREFETCH
#define DPF_SCAN_M4_PREFETCH 1  // 4-record groups in flight per wave
#endif
#ifndef DPF_SCAN_M4_READ_BATCH
#define DPF_SCAN_M4_READ_BATCH 16  // ds_read_b128 issued back to back
#endif

// Cross-tile record prefetch (DPF_SCAN_M4_XTILE, default on): a wave's
// register queue of prefetched records runs across its tiles — the last steps
// of a tile load the first records of the wave's next tile (and the next
// tile's selection block is loaded at the start of the current one), so a
// tile starts with its records in flight instead of waiting one HBM latency,
// and no record is read twice.  (Off: the last steps re-read the tile's own
// first records, 8 records per 128 = 6 % more HBM reads, r03w_pmc.json:
// 19.32 GB read for 17.72 GB algorithmic at Q = 64.)
#ifndef DPF_SCAN_M4_XTILE
#define DPF_SCAN_M4_XTILE 1
#endif
#ifndef DPF_SCAN_M4_SKIP_IDLE
#define DPF_SCAN_M4_SKIP_IDLE 1  // P = 1: lanes without a query skip their row reads
#endif

// The buffer resource of one 128-record tile, based at the tile.  The record
// offset goes in voffset, which the range check covers: the last, partial
// tile limits the range to the bytes left after its base, so records past
// num_records read as zero, and lanes past the slice's width use an offset
// beyond any range.  A tile past the end gets an empty range (its loads
// return zero without touching memory).  (One code path for full and
// partial tiles: two inlined copies made the compiler keep two copies of the
// accumulators, 163 VGPRs instead of ~100.)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t M4TileRsrc(const ScanArgs& a, int64_t tile,
                                                            int dw_lo) {
  const int rec_dwords = a.C * 4;
  const int64_t rec0 = tile << 7;
  if (rec0 >= a.num_records)
    return __builtin_amdgcn_make_buffer_rsrc((void*)a.db, 0, 0, 0x00020000);
  const bool full = rec0 + 128 <= a.num_records;
  const uint32_t* base = reinterpret_cast<const uint32_t*>(a.db) + rec0 * rec_dwords + dw_lo;
  const int64_t left = (a.num_records - rec0) * rec_dwords * 4 - dw_lo * 4;
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, full ? 0x7fffffff : (int)left,
                                           0x00020000);
}

// record r (< 128) of the tile behind `rs`, dword `lane` of the slice
// (record offsets stay below 128 * rec_bytes <= 2^27, see UseScanM4)
__device__ __forceinline__ uint32_t M4Load(__amdgpu_buffer_rsrc_t rs, int voff, int rec_bytes,
                                           bool col_ok, int r) {
  return __builtin_amdgcn_raw_buffer_load_b32(rs, col_ok ? voff + r * rec_bytes : voff, 0, 2);
}

// Prefetch slot idx of a step: record idx of this tile, or (idx >= 128, the
// last steps) record idx - 128 of the next tile — or, without XTILE, the
// current tile's record idx & 127 again.
__device__ __forceinline__ uint32_t M4Prefetch(__amdgpu_buffer_rsrc_t rs,
                                               __amdgpu_buffer_rsrc_t rn, int voff,
                                               int rec_bytes, bool col_ok, int idx) {
#if DPF_SCAN_M4_XTILE
  return M4Load(idx >= 128 ? rn : rs, voff, rec_bytes, col_ok, idx & 127);
#else
  (void)rn;
  return M4Load(rs, voff, rec_bytes, col_ok, idx & 127);
#endif
}

// One 128-record tile, 4 records per step, one table per wave.  `xq` holds
// the tile's first 4 * PF records on entry (prefetched) and the next tile's on
// return.
constexpr int kM4Prefetch = DPF_SCAN_M4_PREFETCH;
template <int P>
__device__ __forceinline__ void ScanM4Tile(uint4 s, __amdgpu_buffer_rsrc_t rs,
                                           __amdgpu_buffer_rsrc_t rn, int voff, int rec_bytes,
                                           bool col_ok, uint32_t (&xq)[4 * kM4Prefetch],
                                           uint32_t (&acc)[64 / P], uint32_t* t, int lane,
                                           int cpart) {
  constexpr int CPL = 16 / P;
  constexpr int ROW = 17;
  // records of the next PF groups in flight (a rotating register queue)
  constexpr int PF = kM4Prefetch;
  // step k: records 4k..4k+3, table row e
  auto step = [&](int k, int e) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t x[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = xq[i];
#pragma unroll
    for (int i = 0; i < 4 * (PF - 1); ++i) xq[i] = xq[i + 4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      xq[4 * (PF - 1) + i] = M4Prefetch(rs, rn, voff, rec_bytes, col_ok, 4 * (k + PF) + i);
    const uint32_t x01 = x[0] ^ x[1], x012 = x01 ^ x[2];
    const uint32_t r[16] = {0u,          x[0],        x[1],        x01,
                            x[2],        x[0] ^ x[2], x[1] ^ x[2], x012,
                            x[3],        x[0] ^ x[3], x[1] ^ x[3], x01 ^ x[3],
                            x[2] ^ x[3], x[0] ^ x[2] ^ x[3], x[1] ^ x[2] ^ x[3], x012 ^ x[3]};
#if DPF_SCAN_M4_ADDTID
    // ds_write_addtid_b32 (address = M0 + offset + 4 * lane): no address
    // VGPRs and half the LDS transfer cycles of ds_write_b32.  The table
    // base is bound to M0 as an "{m0}" input operand, so the compiler writes
    // M0 itself and knows its value at every point.  Its hazard recognizer
    // does not see inside the asm, so the wait state an add-TID op needs
    // after an SALU write of M0 is explicit (without it, rows were written
    // elsewhere at random: nondeterministic 2^26-record scans,
    // tools/diag_scan_determinism.py).
    asm volatile(
        "s_nop 0\n\t"  // SALU write of M0 -> LDS add-TID op: 1 wait state
        "ds_write_addtid_b32 %0 offset:272\n\tds_write_addtid_b32 %1 offset:544\n\t"
        "ds_write_addtid_b32 %2 offset:816\n\tds_write_addtid_b32 %3 offset:1088\n\t"
        "ds_write_addtid_b32 %4 offset:1360\n\tds_write_addtid_b32 %5 offset:1632\n\t"
        "ds_write_addtid_b32 %6 offset:1904\n\tds_write_addtid_b32 %7 offset:2176\n\t"
        "ds_write_addtid_b32 %8 offset:2448\n\tds_write_addtid_b32 %9 offset:2720\n\t"
        "ds_write_addtid_b32 %10 offset:2992\n\tds_write_addtid_b32 %11 offset:3264\n\t"
        "ds_write_addtid_b32 %12 offset:3536\n\tds_write_addtid_b32 %13 offset:3808\n\t"
        "ds_write_addtid_b32 %14 offset:4080"
        :
        : "v"(r[1]), "v"(r[2]), "v"(r[3]), "v"(r[4]), "v"(r[5]), "v"(r[6]), "v"(r[7]),
          "v"(r[8]), "v"(r[9]), "v"(r[10]), "v"(r[11]), "v"(r[12]), "v"(r[13]), "v"(r[14]),
          "v"(r[15]), "{m0}"((uint32_t)(uintptr_t)t)
        : "memory");
    static_assert(ROW * 16 == 272, "addtid offsets assume 272-byte rows");
#else
#pragma unroll
    for (int e = 1; e < 16; ++e) t[e * ROW * 4 + lane] = r[e];
#endif
    // The rows were written by other lanes of this wave, and the next group
    // overwrites them after these reads: LDS executes a wave's operations in
    // issue order, so only compiler motion is fenced (here and at the top).
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint4* row = reinterpret_cast<const uint4*>(t) + e * ROW + cpart * CPL;
    // row reads in batches of RB (their destination VGPRs are what bounds
    // the wave's register budget)
    constexpr int RB = CPL < DPF_SCAN_M4_READ_BATCH ? CPL : DPF_SCAN_M4_READ_BATCH;
#pragma unroll
    for (int c0 = 0; c0 < CPL; c0 += RB) {
#pragma unroll
      for (int c = c0; c < c0 + RB; ++c) {
        const uint4 v = row[c];
        acc[4 * c] ^= v.x;
        acc[4 * c + 1] ^= v.y;
        acc[4 * c + 2] ^= v.z;
        acc[4 * c + 3] ^= v.w;
      }
      if (RB < CPL) __builtin_amdgcn_sched_barrier(0);
    }
  };
  if constexpr (!DPF_SCAN_M4_WORD_LOOPS) {
#pragma unroll 1
    for (int k = 0; k < 32; ++k) step(k, (SelWord(s, k >> 3) >> (4 * (k & 7))) & 15);
  } else {
    // One loop per selection word, two steps per iteration: a word picked by
    // the step index made the compiler lower the pick to a branch tree,
    // split the loop and copy the prefetched registers at the back edge
    // behind an s_waitcnt vmcnt(0) — every step then waited for its own
    // prefetch, one HBM latency per 4 records.
#pragma unroll
    for (int wi = 0; wi < 4; ++wi) {
      const uint32_t word = wi == 0 ? s.x : wi == 1 ? s.y : wi == 2 ? s.z : s.w;
#pragma unroll 2
      for (int kk = 0; kk < 8; ++kk) step(wi * 8 + kk, (word >> (4 * kk)) & 15);
    }
  }
}

// Two 4-record groups per step, each with its own table (tables A and B,
// 4352 bytes apart), so every accumulator takes both selected rows in one
// three-input XOR (gfx950 v_bitop3_b32): the VALU work per group halves
// (64 accumulator XORs per 8 records instead of per 4) while the LDS work
// stays 15 row stores + one row read per query per group.
#ifndef DPF_SCAN_M4_DUAL
#define DPF_SCAN_M4_DUAL 1
#endif
#ifndef DPF_SCAN_M4_DUAL_PF
#define DPF_SCAN_M4_DUAL_PF 1  // steps of 8 records in flight per wave at P = 2
#endif
#ifndef DPF_SCAN_M4_DUAL_RB
#define DPF_SCAN_M4_DUAL_RB 4  // row-pair reads in flight (8 VGPRs each)
#endif
__device__ __forceinline__ uint32_t Xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Stores rows 1..15 of the table at M0 + `base` from the 4 record slices.
#define DPF_M4_STORE_TABLE(base, x)                                                       \
  do {                                                                                    \
    const uint32_t x01 = x[0] ^ x[1], x02 = x[0] ^ x[2], x12 = x[1] ^ x[2];              \
    const uint32_t x03 = x[0] ^ x[3], x13 = x[1] ^ x[3], x23 = x[2] ^ x[3];              \
    const uint32_t x012 = Xor3(x[0], x[1], x[2]), x013 = Xor3(x[0], x[1], x[3]);         \
    const uint32_t x023 = Xor3(x[0], x[2], x[3]), x123 = Xor3(x[1], x[2], x[3]);         \
    const uint32_t x0123 = x01 ^ x23;                                                     \
    asm volatile(                                                                         \
        "s_nop 0\n\t"                                                                     \
        "ds_write_addtid_b32 %0 offset:" #base "+272\n\t"                                 \
        "ds_write_addtid_b32 %1 offset:" #base "+544\n\t"                                 \
        "ds_write_addtid_b32 %2 offset:" #base "+816\n\t"                                 \
        "ds_write_addtid_b32 %3 offset:" #base "+1088\n\t"                                \
        "ds_write_addtid_b32 %4 offset:" #base "+1360\n\t"                                \
        "ds_write_addtid_b32 %5 offset:" #base "+1632\n\t"                                \
        "ds_write_addtid_b32 %6 offset:" #base "+1904\n\t"                                \
        "ds_write_addtid_b32 %7 offset:" #base "+2176\n\t"                                \
        "ds_write_addtid_b32 %8 offset:" #base "+2448\n\t"                                \
        "ds_write_addtid_b32 %9 offset:" #base "+2720\n\t"                                \
        "ds_write_addtid_b32 %10 offset:" #base "+2992\n\t"                               \
        "ds_write_addtid_b32 %11 offset:" #base "+3264\n\t"                               \
        "ds_write_addtid_b32 %12 offset:" #base "+3536\n\t"                               \
        "ds_write_addtid_b32 %13 offset:" #base "+3808\n\t"                               \
        "ds_write_addtid_b32 %14 offset:" #base "+4080"                                   \
        :                                                                                 \
        : "v"(x[0]), "v"(x[1]), "v"(x01), "v"(x[2]), "v"(x02), "v"(x12), "v"(x012),      \
          "v"(x[3]), "v"(x03), "v"(x13), "v"(x013), "v"(x23), "v"(x023), "v"(x123),       \
          "v"(x0123), "{m0}"((uint32_t)(uintptr_t)t)                                      \
        : "memory");                                                                      \
  } while (0)

// the next DPF steps' records (8 each) in flight at P = 2
constexpr int M4DualPrefetch(int P) { return P == 2 ? DPF_SCAN_M4_DUAL_PF : 1; }

// LDS / VALU query split of the P = 1 pass (A/B experiment, DESIGN.md §3.5,
// default 0 = off): with more than 48 queries in the pass, the queries of
// the fourth lane group (48-63) take no table rows — that group's
// ds_read_b128 work leaves the LDS — and are summed on the VALU instead, in
// the lane = dword layout the records arrive in: accm[j] ^= x_i & mask, the
// mask from query 48 + j's selection byte (v_readlane from its lane).
#ifndef DPF_SCAN_M4_VALU_Q
#define DPF_SCAN_M4_VALU_Q 0
#endif
static_assert(DPF_SCAN_M4_VALU_Q == 0 || DPF_SCAN_M4_VALU_Q == 16, "VALU queries: 0 or 16");
#ifndef DPF_SCAN_M4_VALU_MASK
#define DPF_SCAN_M4_VALU_MASK 0  // 1: the per-record masks computed on the VALU
#endif
constexpr int kM4ValuQ = DPF_SCAN_M4_VALU_Q;
constexpr int kM4TableQ = 64 - kM4ValuQ;
// lanes of the fourth group (upper half, lanes 4-11 / 16-19 / 28-31) in
// query order (M4LaneMap<1> with SKIP_IDLE): query 48 + j sits in lane
// kM4Group3Lane[j]
__device__ __forceinline__ int M4Group3Lane(int j) {
  return 32 + (j < 8 ? 4 + j : j < 12 ? 16 + (j - 8) : 28 + (j - 12));
}

template <int P>
__device__ __forceinline__ void ScanM4Tile2(uint4 s, __amdgpu_buffer_rsrc_t rs,
                                            __amdgpu_buffer_rsrc_t rn, int voff, int rec_bytes,
                                            bool col_ok, uint32_t (&xq)[8 * M4DualPrefetch(P)],
                                            uint32_t (&acc)[64 / P], uint32_t* t, int cpart,
                                            bool q_ok, uint32_t (&accm)[kM4ValuQ > 0 ? kM4ValuQ : 1],
                                            bool valu_pass) {
  constexpr int CPL = 16 / P;
  constexpr int ROW = 17;
  constexpr int DPF = M4DualPrefetch(P);
  // step k: records 8k..8k+7 into tables A and B, selection byte sb
  auto step = [&](int k, uint32_t sb) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t xa[4], xb[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      xa[i] = xq[i];
      xb[i] = xq[4 + i];
    }
#pragma unroll
    for (int i = 0; i < 8 * (DPF - 1); ++i) xq[i] = xq[i + 8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
      xq[8 * (DPF - 1) + i] = M4Prefetch(rs, rn, voff, rec_bytes, col_ok, 8 * (k + DPF) + i);
    DPF_M4_STORE_TABLE(0, xa);
    DPF_M4_STORE_TABLE(4352, xb);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if constexpr (P == 1 && kM4ValuQ > 0) {
      if (valu_pass) {  // wave-uniform: queries 48-63 on the VALU, every lane
#pragma unroll
        for (int j = 0; j < kM4ValuQ; ++j) {
          uint32_t sbj = __builtin_amdgcn_readlane(sb, M4Group3Lane(j));
#if DPF_SCAN_M4_VALU_MASK
          // the masks on the VALU (the scalar unit is shared by the CU's SIMDs)
          asm volatile("v_mov_b32 %0, %1" : "=v"(sbj) : "s"(sbj));
#endif
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const uint32_t m = 0u - ((sbj >> i) & 1u);
            accm[j] = __builtin_amdgcn_bitop3_b32(accm[j], i < 4 ? xa[i] : xb[i - 4], m, 0x78);
          }
        }
      }
    }
    // groups 2k and 2k + 1: low nibble for table A
    if (P == 1 && DPF_SCAN_M4_SKIP_IDLE && !q_ok) return;  // an idle lane reads nothing
    const uint4* ra = reinterpret_cast<const uint4*>(t) + (sb & 15) * ROW + cpart * CPL;
    const uint4* rb = reinterpret_cast<const uint4*>(t) + (16 + (sb >> 4)) * ROW + cpart * CPL;
    constexpr int RB = CPL < DPF_SCAN_M4_DUAL_RB ? CPL : DPF_SCAN_M4_DUAL_RB;
#pragma unroll
    for (int c0 = 0; c0 < CPL; c0 += RB) {
#pragma unroll
      for (int c = c0; c < c0 + RB; ++c) {
        const uint4 v = ra[c], w = rb[c];
        acc[4 * c] = Xor3(acc[4 * c], v.x, w.x);
        acc[4 * c + 1] = Xor3(acc[4 * c + 1], v.y, w.y);
        acc[4 * c + 2] = Xor3(acc[4 * c + 2], v.z, w.z);
        acc[4 * c + 3] = Xor3(acc[4 * c + 3], v.w, w.w);
      }
      if (RB < CPL) __builtin_amdgcn_sched_barrier(0);
    }
  };
  if constexpr ((P == 1 && DPF_SCAN_M4_WORD_LOOPS < 2) || !DPF_SCAN_M4_WORD_LOOPS) {
    // (P = 1 at 126 VGPRs: the two-step word loops below spill)
#pragma unroll 1
    for (int k = 0; k < 16; ++k) step(k, (SelWord(s, k >> 2) >> (8 * (k & 3))) & 255);
  } else {
    // one loop per selection word, two steps per iteration (see ScanM4Tile)
#pragma unroll
    for (int wi = 0; wi < 4; ++wi) {
      const uint32_t word = wi == 0 ? s.x : wi == 1 ? s.y : wi == 2 ? s.z : s.w;
#pragma unroll 2
      for (int kk = 0; kk < 4; ++kk) step(wi * 4 + kk, (word >> (8 * kk)) & 255);
    }
  }
}

#ifndef DPF_SCAN_M4_P4_WAVES
#define DPF_SCAN_M4_P4_WAVES 8  // 8192 parts = one resident round at 8 waves/SIMD
#endif

// Lane -> (query of the wave, column part).  A ds_read_b128 is served in four
// 16-lane groups, {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31} and the same
// two in the upper half (MI355X_MICROARCH.md §LDS).  Lanes of one group that
// read the same column of different rows hit different slots ((e + c) mod 16)
// and lanes reading the same row broadcast, but lanes of one group reading
// different columns of different rows can collide.  P = 1 and 2 put one part
// in each group with part = lane / QW; at P = 4 that puts two parts in each
// group (`SQ_LDS_BANK_CONFLICT` 2.6e8 cycles per Q = 16 launch, 19 % of the
// kernel), so there part = the lane's group and the query its rank in it.
#ifndef DPF_SCAN_M4_P4_GROUPS
#define DPF_SCAN_M4_P4_GROUPS 1
#endif
template <int P>
__device__ __forceinline__ void M4LaneMap(int lane, int& ql, int& cpart) {
  constexpr int QW = 64 / P;
  if constexpr (P == 4 && DPF_SCAN_M4_P4_GROUPS) {
    constexpr uint32_t kGroupB = 0xF00F0FF0u;  // lanes 4-11, 16-19, 28-31 of a half
    const int m = lane & 31;
    const uint32_t in_b = (kGroupB >> m) & 1u;
    const uint32_t g = in_b ? kGroupB : ~kGroupB;
    cpart = 2 * (lane >> 5) + (int)in_b;
    ql = __builtin_popcount(g & ((1u << m) - 1u));
  } else if constexpr (P == 1 && DPF_SCAN_M4_SKIP_IDLE) {
    // queries fill the four lane groups in order (16 per group), so a pass of
    // up to 48 queries leaves a whole group idle — and its lanes, which skip
    // their row reads, cost the LDS nothing (row reads of lanes without a
    // query used to read row 0: Q = 33 took as long as Q = 64)
    constexpr uint32_t kGroupB = 0xF00F0FF0u;
    const int m = lane & 31;
    const uint32_t in_b = (kGroupB >> m) & 1u;
    const uint32_t g = in_b ? kGroupB : ~kGroupB;
    ql = 16 * (2 * (lane >> 5) + (int)in_b) + __builtin_popcount(g & ((1u << m) - 1u));
    cpart = 0;
  } else {
    ql = lane % QW;
    cpart = lane / QW;
  }
}
#ifndef DPF_SCAN_M4_P1_WAVES
#define DPF_SCAN_M4_P1_WAVES 4  // 100 VGPRs (5 waves: 4 spilled, Q = 64 4.31 vs 4.36 ms)
#endif
template <int P>
__global__ __launch_bounds__(kScanM4Block, P == 1 ? DPF_SCAN_M4_P1_WAVES : P == 2 ? 4 : DPF_SCAN_M4_P4_WAVES)
void KPirScanM4(ScanArgs a) {
  constexpr int QW = 64 / P;        // queries per wave
  constexpr int CPL = 16 / P;       // 16-byte columns of the slice per lane
  constexpr int ROW = 17;           // uint4 per table row (272 B)
  // (P = 4 keeps one table: two would cap it at 4 waves/SIMD by LDS)
  constexpr bool DUAL = DPF_SCAN_M4_DUAL && P <= 2;
  constexpr int TABLES = DUAL ? 2 : 1;
  __shared__ uint4 tab[kScanM4Waves][TABLES * 16 * ROW];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // qgroups = 2 (P = 1, 65-128 queries): the waves of a pair scan the same
  // tiles for queries [0, 64) and [64, 128), each with its own table — one
  // pass over the rows instead of two, no barrier (the pair's second loads
  // of a tile mostly hit in cache).
  const int qg = a.qgroups;
  int64_t pb;
  int slice;
  M4BlockSlice(a, pb, slice);
  const int64_t part = pb * (kScanM4Waves / qg) + wave / qg;
  if (part >= a.parts) return;  // wave-uniform; no block barrier below
  int ql, cpart;
  M4LaneMap<P>(lane, ql, cpart);
  const int q = (wave % qg) * QW + ql;
  const int dw_lo = slice * 64;
  const int width = min(64, a.C * 4 - dw_lo);  // dwords of this slice
  const bool col_ok = lane < width;
  const bool q_ok = q < a.nq;
  // the VALU split (P = 1, more than 48 queries): lanes of queries 48-63
  // load their selection blocks (read by v_readlane) but take no table rows
  const bool valu_pass = P == 1 && DUAL && kM4ValuQ > 0 && a.nq > kM4TableQ;
  const bool q_tab = q_ok && !(valu_pass && ql >= kM4TableQ);
  uint32_t accm[kM4ValuQ > 0 ? kM4ValuQ : 1];
#pragma unroll
  for (int j = 0; j < (kM4ValuQ > 0 ? kM4ValuQ : 1); ++j) accm[j] = 0u;
  uint32_t* t = reinterpret_cast<uint32_t*>(tab[wave]);
  t[lane] = 0u;  // row 0 (no record selected) stays zero
  if (TABLES == 2) t[16 * ROW * 4 + lane] = 0u;
  uint32_t acc[4 * CPL];
#pragma unroll
  for (int i = 0; i < 4 * CPL; ++i) acc[i] = 0u;
  const int64_t tiles = (a.num_records + 127) >> 7;
  const int rec_bytes = a.C * 16;
  const int voff = col_ok ? lane * 4 : (int)0x80000000u;
  constexpr int XQ = DUAL ? 8 * M4DualPrefetch(P) : 4 * kM4Prefetch;
  int64_t tile = part;
  if (tile < tiles) {  // wave-uniform
    __amdgpu_buffer_rsrc_t rs = M4TileRsrc(a, tile, dw_lo);
    uint4 s = q_ok ? a.sel[(int64_t)(a.q0 + q) * a.sel_blocks + tile] : make_uint4(0, 0, 0, 0);
    uint32_t xq[XQ];
#pragma unroll
    for (int i = 0; i < XQ; ++i) xq[i] = M4Load(rs, voff, rec_bytes, col_ok, i);
    const int64_t n_it = (tiles - part + a.parts - 1) / a.parts;
    for (;;) {
      ScanPrio<DPF_SCAN_M4_PRIO != 0>((tile - part) / a.parts, n_it);
      const int64_t next = tile + a.parts;
      const bool more = next < tiles;
      // the next tile's resource (an empty range past the end) and selection
      // block, in flight while this tile runs
      const __amdgpu_buffer_rsrc_t rn = M4TileRsrc(a, next, dw_lo);
      const uint4 sn = (q_ok && more) ? a.sel[(int64_t)(a.q0 + q) * a.sel_blocks + next]
                                      : make_uint4(0, 0, 0, 0);
      if constexpr (DUAL)
        ScanM4Tile2<P>(s, rs, rn, voff, rec_bytes, col_ok, xq, acc, t, cpart, q_tab, accm,
                       valu_pass);
      else
        ScanM4Tile<P>(s, rs, rn, voff, rec_bytes, col_ok, xq, acc, t, lane, cpart);
      if (!more) break;
      tile = next;
      rs = rn;
      s = sn;
    }
  }
  if constexpr (P == 1 && kM4ValuQ > 0) {
    if (valu_pass) {  // dword `lane` of the slice of each VALU query
      for (int j = 0; j < kM4ValuQ && kM4TableQ + j < a.nq; ++j) {
        uint32_t* o = reinterpret_cast<uint32_t*>(
            a.partials + (part * a.total_q + a.q0 + kM4TableQ + j) * a.C + slice * 16);
        if (col_ok) o[lane] = accm[j];
      }
    }
  }
  if (!q_tab) return;
  // this lane's columns [cpart * CPL, +CPL) of the slice, clipped to the record
  uint4* out = a.partials + (part * a.total_q + a.q0 + q) * a.C + slice * 16;
  const int chunks = (width + 3) / 4;
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int col = cpart * CPL + c;
    if (col < chunks)
      out[col] = make_uint4(acc[4 * c], acc[4 * c + 1], acc[4 * c + 2], acc[4 * c + 3]);
  }
}

// 65-128 queries, one wave pair per block sharing its tables: per step of 8
// records wave w loads records 4w..4w+3 and builds table w (A or B) only,
// one barrier publishes both, and each wave reads rows from both for its 64
// queries.  Tables are double-buffered (step parity), so a wave overwrites a
// buffer only after passing the next step's barrier, which its partner
// reaches after finishing its reads of that buffer.  Against two private
// table pairs this halves the row stores and the record loads per step.
#ifndef DPF_SCAN_M4_SHARED
#define DPF_SCAN_M4_SHARED 1
#endif
#ifndef DPF_SCAN_M4_PAIR_RB
#define DPF_SCAN_M4_PAIR_RB 4  // row pairs in flight (118 VGPRs; 2: 102, Q = 100 6.11 vs 6.03 ms)
#endif
#ifndef DPF_SCAN_M4_PAIR_WAVES
#define DPF_SCAN_M4_PAIR_WAVES 4
#endif
constexpr int kScanM4PairBlock = 128;

__device__ __forceinline__ void ScanM4PairStep(const uint32_t (&x)[4], uint32_t sb, int buf,
                                               uint32_t* t0, const uint4* tab0,
                                               uint32_t (&acc)[64], bool q_ok) {
  constexpr int ROW = 17;
  // this wave's table in buffer `buf` (M0 = its base; buffer 1 is 8704 B on)
  uint32_t* t = t0 + buf * (2 * 16 * ROW * 4);
  DPF_M4_STORE_TABLE(0, x);
  // LDS-only barrier: the tables are published, the next step's record loads
  // stay in flight (__syncthreads would also wait for them, vmcnt(0))
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  if (DPF_SCAN_M4_SKIP_IDLE && !q_ok) return;  // an idle lane reads nothing
  const uint4* ra = tab0 + (2 * buf) * 16 * ROW + (sb & 15) * ROW;
  const uint4* rb = tab0 + (2 * buf + 1) * 16 * ROW + (sb >> 4) * ROW;
  constexpr int RB = DPF_SCAN_M4_PAIR_RB;
#pragma unroll
  for (int c0 = 0; c0 < 16; c0 += RB) {
#pragma unroll
    for (int c = c0; c < c0 + RB; ++c) {
      const uint4 v = ra[c], w = rb[c];
      acc[4 * c] = Xor3(acc[4 * c], v.x, w.x);
      acc[4 * c + 1] = Xor3(acc[4 * c + 1], v.y, w.y);
      acc[4 * c + 2] = Xor3(acc[4 * c + 2], v.z, w.z);
      acc[4 * c + 3] = Xor3(acc[4 * c + 3], v.w, w.w);
    }
    if (RB < 16) __builtin_amdgcn_sched_barrier(0);
  }
}

__global__ __launch_bounds__(kScanM4PairBlock, DPF_SCAN_M4_PAIR_WAVES)
void KPirScanM4Pair(ScanArgs a) {
  constexpr int ROW = 17;
  // [buffer][table A/B][row]: wave w writes table w of each buffer
  __shared__ uint4 tab[2][2][16 * ROW];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int64_t part;  // block-uniform: both waves take the barriers
  int slice;
  M4BlockSlice(a, part, slice);
  int ql, cpart;
  M4LaneMap<1>(lane, ql, cpart);  // queries fill whole lane groups (idle groups skip reads)
  const int q = wave * 64 + ql;
  const int dw_lo = slice * 64;
  const int width = min(64, a.C * 4 - dw_lo);
  const bool col_ok = lane < width;
  const bool q_ok = q < a.nq;
  uint32_t* t = reinterpret_cast<uint32_t*>(tab[0][wave]);
  const uint4* tab0 = &tab[0][0][0];
  t[lane] = 0u;                  // row 0 of this wave's table, buffer 0
  t[2 * 16 * ROW * 4 + lane] = 0u;  // and buffer 1
  uint32_t acc[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) acc[i] = 0u;
  const int64_t tiles = (a.num_records + 127) >> 7;
  const int rec_bytes = a.C * 16;
  const int voff = col_ok ? lane * 4 : (int)0x80000000u;
  int64_t tile = part;
  if (tile < tiles) {  // block-uniform
    __amdgpu_buffer_rsrc_t rs = M4TileRsrc(a, tile, dw_lo);
    uint4 s = q_ok ? a.sel[(int64_t)(a.q0 + q) * a.sel_blocks + tile] : make_uint4(0, 0, 0, 0);
    // this wave's 4 records of the next step in flight (across tiles)
    uint32_t xq[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) xq[i] = M4Load(rs, voff, rec_bytes, col_ok, 4 * wave + i);
    const int64_t n_it = (tiles - part + a.parts - 1) / a.parts;
    for (;;) {
      ScanPrio((tile - part) / a.parts, n_it);
      const int64_t next = tile + a.parts;
      const bool more = next < tiles;
      const __amdgpu_buffer_rsrc_t rn = M4TileRsrc(a, next, dw_lo);
      const uint4 sn = (q_ok && more) ? a.sel[(int64_t)(a.q0 + q) * a.sel_blocks + next]
                                      : make_uint4(0, 0, 0, 0);
#pragma unroll 1
      for (int k = 0; k < 16; ++k) {
        uint32_t x[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          x[i] = xq[i];
          xq[i] = M4Prefetch(rs, rn, voff, rec_bytes, col_ok, 8 * (k + 1) + 4 * wave + i);
        }
        ScanM4PairStep(x, (SelWord(s, k >> 2) >> (8 * (k & 3))) & 255, k & 1, t, tab0, acc,
                       q_ok);
      }
      if (!more) break;
      tile = next;
      rs = rn;
      s = sn;
    }
  }
  if (!q_ok) return;
  uint4* out = a.partials + (part * a.total_q + a.q0 + q) * a.C + slice * 16;
  const int chunks = (width + 3) / 4;
#pragma unroll
  for (int c = 0; c < 16; ++c)
    if (c < chunks)
      out[c] = make_uint4(acc[4 * c], acc[4 * c + 1], acc[4 * c + 2], acc[4 * c + 3]);
}

#ifndef DPF_SCAN_M4_PAIRS
#define DPF_SCAN_M4_PAIRS 1  // wave pairs for 65-128 queries (else 64 per pass)
#endif
int PirScanM4Queries(int rem) {
  return std::min(rem, (DPF_SCAN_M4_PAIRS && rem > 64) ? 128 : rem > 32 ? 64 : rem > 16 ? 32 : 16);
}

int LaunchPirScanM4(int nq, int parts, int slices, hipStream_t st, const ScanArgs& args) {
  const int P = nq > 32 ? 1 : nq > 16 ? 2 : 4;
  ScanArgs a = args;
  a.qgroups = nq > 64 ? 2 : 1;
  a.slice_major = (DPF_SCAN_M4_SLICE_MAJOR && slices > 1) ? 1 : 0;
  const int per_block = kScanM4Waves / a.qgroups;
  const dim3 g = a.slice_major ? dim3(((parts + per_block - 1) / per_block) * slices, 1)
                               : dim3((parts + per_block - 1) / per_block, slices);
  if (DPF_SCAN_M4_SHARED && a.qgroups == 2) {
    const dim3 gp = a.slice_major ? dim3(parts * slices, 1) : dim3(parts, slices);
    hipLaunchKernelGGL(KPirScanM4Pair, gp, dim3(kScanM4PairBlock), 0, st, a);
  } else if (P == 1)
    hipLaunchKernelGGL((KPirScanM4<1>), g, dim3(kScanM4Block), 0, st, a);
  else if (P == 2)
    hipLaunchKernelGGL((KPirScanM4<2>), g, dim3(kScanM4Block), 0, st, a);
  else
    hipLaunchKernelGGL((KPirScanM4<4>), g, dim3(kScanM4Block), 0, st, a);
  return LaunchCheck("pir scan kernel launch");
}

int LaunchGatherRows(int grid, hipStream_t st, int64_t n, const int64_t* src_offset,
                     int64_t opp, int64_t stride, const char* in, char* out, int64_t in_rows,
                     int* err) {
  // Row offsets are multiples of opp rows; with (opp x stride) % 16 == 0 and
  // 16-byte-aligned buffers every segment is whole 16-byte words.
  if ((opp * stride) % 16 == 0 && (uintptr_t)in % 16 == 0 && (uintptr_t)out % 16 == 0 &&
      (opp * stride) / 16 > 0 && stride % 16 == 0) {
    hipLaunchKernelGGL(KGatherRows16, dim3(grid), dim3(256), 0, st, n, src_offset,
                       opp * stride / 16, stride / 16, (const uint4*)in, (uint4*)out, opp,
                       in_rows, err);
  } else if ((opp * stride) % 16 == 0 && (uintptr_t)in % 16 == 0 && (uintptr_t)out % 16 == 0 &&
             (16 % stride) == 0) {
    hipLaunchKernelGGL(KGatherRowsSmall, dim3(grid), dim3(256), 0, st, n, src_offset,
                       opp * stride / 16, 16 / stride, (const uint4*)in, (uint4*)out, opp,
                       in_rows, err);
  } else {
    hipLaunchKernelGGL(KGatherRows, dim3(grid), dim3(256), 0, st, n, src_offset, opp, stride,
                       in, out, in_rows, err);
  }
  return LaunchCheck("gather kernel launch");
}

int LaunchXorFold(unsigned blocks, hipStream_t st, const uint4* parts, int num_parts,
                  int64_t words, uint4* out, uint4* clear) {
  hipLaunchKernelGGL(KXorFold, dim3(blocks), dim3(256), 0, st, parts, num_parts, words, out,
                     clear);
  return LaunchCheck("xor fold kernel launch");
}

int LaunchXorFoldBytes(int grid, hipStream_t st, const uint8_t* parts, int num_parts,
                       int64_t bytes, uint8_t* out) {
  hipLaunchKernelGGL(KXorFoldBytes, dim3(grid), dim3(256), 0, st, parts, num_parts, bytes,
                     out);
  return LaunchCheck("xor fold kernel launch");
}

template <int G>
static void LaunchScanG(int nq, dim3 g, hipStream_t st, const ScanArgs& a) {
  if (G == 1 && DPF_SCAN_G1_SLICE_MAJOR) g = dim3(g.x * g.y, 1);  // slice = block % slices
  if (nq == 1)
    hipLaunchKernelGGL((KPirScanG<1, G>), g, dim3(kScanBlock), 0, st, a);
  else if (nq <= 2)
    hipLaunchKernelGGL((KPirScanG<2, G>), g, dim3(kScanBlock), 0, st, a);
  else if (nq <= 4)
    hipLaunchKernelGGL((KPirScanG<4, G>), g, dim3(kScanBlock), 0, st, a);
  else if (nq <= 8)
    hipLaunchKernelGGL((KPirScanG<8, G>), g, dim3(kScanBlock), 0, st, a);
  else
    hipLaunchKernelGGL((KPirScanG<16, G>), g, dim3(kScanBlock), 0, st, a);
}

int PirScanGroup(int C) {
  if (C > 32) return 1;
  int g = 1;
  while (g * 2 * C <= 64) g *= 2;
  return g;
}

int LaunchPirScan(int nq, dim3 g, hipStream_t st, const ScanArgs& a) {
  switch (PirScanGroup(a.C)) {
    case 1:
      LaunchScanG<1>(nq, g, st, a);
      break;
    case 2:
      LaunchScanG<2>(nq, g, st, a);
      break;
    case 4:
      LaunchScanG<4>(nq, g, st, a);
      break;
    case 8:
      LaunchScanG<8>(nq, g, st, a);
      break;
    case 16:
      LaunchScanG<16>(nq, g, st, a);
      break;
    case 32:
      LaunchScanG<32>(nq, g, st, a);
      break;
    default:
      LaunchScanG<64>(nq, g, st, a);
  }
  return LaunchCheck("pir scan kernel launch");
}

}  // namespace dpf_amd
