// k_incremental.hip — EvaluateUntil's prefix bookkeeping on the device
// (dpf/distributed_point_function.h:772-796 de-duplication, cc:374-476
// lookup of the stored partial evaluations), for the device-resident context
// of dpf.cc.
//
// DedupPrefixes: for sorted prefixes, tree index t_i = p_i >> bbits; the
// unique tree indices in order (u = number of distinct t in [0, i] minus one
// is prefix i's unique index), the low bits p_i & (2^bbits - 1), the count,
// and flags: bit 0 the prefixes are not sorted, bit 1 one is >= the limit
// (the previous level's domain size).  Three launches: per-block flag counts,
// one block scanning the counts, per-block writes.
//
// LookupPartialEvaluations: unique tree index u -> the stored partial
// evaluation of u >> shift (binary search in the previous call's strictly
// increasing list) or the key's root; bit 2 of flags when one is missing.
// Either flag sends the caller back to the host path, which produces the
// reference's result or error.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "internal.h"
#include "kernel_args.h"

namespace dpf_amd {
namespace {

struct U128 {
  uint64_t lo, hi;
};

__device__ __forceinline__ bool Less(const U128& a, const U128& b) {
  return a.hi < b.hi || (a.hi == b.hi && a.lo < b.lo);
}
__device__ __forceinline__ bool Equal(const U128& a, const U128& b) {
  return a.hi == b.hi && a.lo == b.lo;
}
__device__ __forceinline__ U128 Shr(const U128& a, int s) {
  if (s <= 0) return a;
  if (s >= 128) return U128{0, 0};
  if (s >= 64) return U128{a.hi >> (s - 64), 0};
  return U128{(a.lo >> s) | (a.hi << (64 - s)), a.hi >> s};
}

constexpr int kDedupBlock = 256;
constexpr int kDedupPer = 8;  // prefixes per thread
constexpr int64_t kDedupChunk = kDedupBlock * kDedupPer;

struct DedupArgs {
  const U128* p;
  int64_t n;
  int bbits;
  int has_limit;
  U128 limit;
  int32_t* pidx;
  uint8_t* plow;
  U128* unique;
  int64_t* count;
  int64_t* block_off;  // [blocks]: flag counts, then their exclusive scan
  int* flags;
};

// Flag of prefix i (a new tree index) and the order / range checks against
// its predecessor.
__device__ __forceinline__ bool NewIndex(const DedupArgs& a, int64_t i, const U128& cur,
                                         int* bad) {
  if (a.has_limit && !Less(cur, a.limit)) *bad |= 2;
  if (i == 0) return true;
  const U128 prev = a.p[i - 1];
  if (Less(cur, prev)) *bad |= 1;
  return !Equal(Shr(cur, a.bbits), Shr(prev, a.bbits));
}

// Block sum of `v` over kDedupBlock threads (wave sums through LDS).
__device__ __forceinline__ int64_t BlockSum(int64_t v, int64_t* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  int64_t s = 0;
  for (int w = 0; w < kDedupBlock / 64; ++w) s += red[w];
  return s;
}

__global__ __launch_bounds__(kDedupBlock) void KDedupCount(DedupArgs a) {
  __shared__ int64_t red[kDedupBlock / 64];
  const int64_t base = (int64_t)blockIdx.x * kDedupChunk + (int64_t)threadIdx.x * kDedupPer;
  int bad = 0;
  int64_t c = 0;
  for (int k = 0; k < kDedupPer; ++k) {
    const int64_t i = base + k;
    if (i < a.n) c += NewIndex(a, i, a.p[i], &bad);
  }
  if (bad) atomicOr(a.flags, bad);
  const int64_t s = BlockSum(c, red);
  if (threadIdx.x == 0) a.block_off[blockIdx.x] = s;
}

// One block: exclusive scan of the per-block counts, total into *count.
__global__ __launch_bounds__(1024) void KDedupScan(int64_t* block_off, int64_t blocks,
                                                   int64_t* count) {
  __shared__ int64_t part[1024];
  int64_t carry = 0;
  for (int64_t b0 = 0; b0 < blocks; b0 += 1024) {
    const int64_t b = b0 + threadIdx.x;
    const int64_t v = b < blocks ? block_off[b] : 0;
    part[threadIdx.x] = v;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {  // inclusive Hillis-Steele scan
      const int64_t add = threadIdx.x >= (unsigned)o ? part[threadIdx.x - o] : 0;
      __syncthreads();
      part[threadIdx.x] += add;
      __syncthreads();
    }
    if (b < blocks) block_off[b] = carry + part[threadIdx.x] - v;
    carry += part[1023];
    __syncthreads();
  }
  if (threadIdx.x == 0) *count = carry;
}

__global__ __launch_bounds__(kDedupBlock) void KDedupWrite(DedupArgs a) {
  __shared__ int64_t scan[kDedupBlock];
  const int64_t base = (int64_t)blockIdx.x * kDedupChunk + (int64_t)threadIdx.x * kDedupPer;
  int bad = 0;
  bool f[kDedupPer];
  U128 cur[kDedupPer];
  int64_t c = 0;
#pragma unroll
  for (int k = 0; k < kDedupPer; ++k) {
    const int64_t i = base + k;
    f[k] = false;
    if (i < a.n) {
      cur[k] = a.p[i];
      f[k] = NewIndex(a, i, cur[k], &bad);
    }
    c += f[k];
  }
  // exclusive scan of the threads' counts (inclusive Hillis-Steele, shifted)
  scan[threadIdx.x] = c;
  __syncthreads();
  for (int o = 1; o < kDedupBlock; o <<= 1) {
    const int64_t add = threadIdx.x >= (unsigned)o ? scan[threadIdx.x - o] : 0;
    __syncthreads();
    scan[threadIdx.x] += add;
    __syncthreads();
  }
  // flags before this thread's first prefix, over the whole list
  int64_t u = a.block_off[blockIdx.x] + scan[threadIdx.x] - c;
  const uint64_t mask = (a.bbits >= 64) ? ~0ull : ((1ull << a.bbits) - 1);
#pragma unroll
  for (int k = 0; k < kDedupPer; ++k) {
    const int64_t i = base + k;
    if (i >= a.n) break;
    if (f[k]) a.unique[u++] = Shr(cur[k], a.bbits);
    a.pidx[i] = (int32_t)(u - 1);
    a.plow[i] = (uint8_t)(cur[k].lo & mask);
  }
}

struct LookupArgs {
  const U128* unique;
  const int64_t* count;
  int64_t n_max;
  int shift;
  int from_root;
  const U128* stored;
  int64_t stored_n;
  const uint4* stored_seeds;
  const uint8_t* stored_cb;
  uint4 root_seed;
  uint32_t root_cb;
  uint4* seeds_out;
  uint8_t* cb_out;
  int* flags;
};

__global__ __launch_bounds__(256) void KLookupPartials(LookupArgs a) {
  const int64_t cnt = *a.count;
  const int64_t m = cnt < a.n_max ? cnt : a.n_max;
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < m; u += step) {
    if (a.from_root) {
      a.seeds_out[u] = a.root_seed;
      a.cb_out[u] = (uint8_t)a.root_cb;
      continue;
    }
    const U128 q = Shr(a.unique[u], a.shift);
    int64_t lo = 0, hi = a.stored_n;  // first stored prefix >= q
    while (lo < hi) {
      const int64_t mid = lo + ((hi - lo) >> 1);
      if (Less(a.stored[mid], q))
        lo = mid + 1;
      else
        hi = mid;
    }
    if (lo < a.stored_n && Equal(a.stored[lo], q)) {
      a.seeds_out[u] = a.stored_seeds[lo];
      a.cb_out[u] = a.stored_cb[lo];
    } else {
      atomicOr(a.flags, 4);
      a.seeds_out[u] = make_uint4(0, 0, 0, 0);
      a.cb_out[u] = 0;
    }
  }
}

}  // namespace

int64_t DedupBlocks(int64_t n) { return (n + kDedupChunk - 1) / kDedupChunk; }

int DedupPrefixes(const void* prefixes, int64_t n, int bbits, const uint64_t* limit,
                  int32_t* pidx, uint8_t* plow, void* unique, int64_t* count,
                  int64_t* block_scratch, int* flags, void* stream) {
  if (n <= 0 || n > INT32_MAX || bbits < 0 || bbits > 127)
    return SetError(DPF_AMD_INTERNAL, "bad prefix de-duplication arguments");
  hipStream_t st = (hipStream_t)stream;
  DedupArgs a;
  a.p = (const U128*)prefixes;
  a.n = n;
  a.bbits = bbits;
  a.has_limit = limit != nullptr;
  a.limit = limit ? U128{limit[0], limit[1]} : U128{0, 0};
  a.pidx = pidx;
  a.plow = plow;
  a.unique = (U128*)unique;
  a.count = count;
  a.block_off = block_scratch;
  a.flags = flags;
  const int64_t blocks = DedupBlocks(n);
  hipLaunchKernelGGL(KDedupCount, dim3((unsigned)blocks), dim3(kDedupBlock), 0, st, a);
  int rc = LaunchCheck("dedup count kernel launch");
  if (rc != DPF_AMD_OK) return rc;
  hipLaunchKernelGGL(KDedupScan, dim3(1), dim3(1024), 0, st, block_scratch, blocks, count);
  rc = LaunchCheck("dedup scan kernel launch");
  if (rc != DPF_AMD_OK) return rc;
  hipLaunchKernelGGL(KDedupWrite, dim3((unsigned)blocks), dim3(kDedupBlock), 0, st, a);
  return LaunchCheck("dedup write kernel launch");
}

int LookupPartialEvaluations(const void* unique, const int64_t* count, int64_t n_max, int shift,
                             const void* stored, int64_t stored_n, const void* stored_seeds,
                             const uint8_t* stored_cb, const uint64_t root_seed[2], int root_cb,
                             bool from_root, void* seeds_out, uint8_t* cb_out, int* flags,
                             void* stream) {
  if (n_max <= 0) return DPF_AMD_OK;
  if (!from_root && (stored_n <= 0 || !stored || !stored_seeds || !stored_cb))
    return SetError(DPF_AMD_INTERNAL, "bad partial-evaluation lookup arguments");
  LookupArgs a;
  a.unique = (const U128*)unique;
  a.count = count;
  a.n_max = n_max;
  a.shift = shift;
  a.from_root = from_root ? 1 : 0;
  a.stored = (const U128*)stored;
  a.stored_n = from_root ? 0 : stored_n;
  a.stored_seeds = (const uint4*)stored_seeds;
  a.stored_cb = stored_cb;
  a.root_seed = make_uint4((uint32_t)root_seed[0], (uint32_t)(root_seed[0] >> 32),
                           (uint32_t)root_seed[1], (uint32_t)(root_seed[1] >> 32));
  a.root_cb = (uint32_t)(root_cb != 0);
  a.seeds_out = (uint4*)seeds_out;
  a.cb_out = cb_out;
  a.flags = flags;
  const int grid = (int)std::min<int64_t>(2048, (n_max + 255) / 256);
  hipLaunchKernelGGL(KLookupPartials, dim3(grid), dim3(256), 0, (hipStream_t)stream, a);
  return LaunchCheck("partial-evaluation lookup kernel launch");
}

}  // namespace dpf_amd
