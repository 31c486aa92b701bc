// expand_device.h — the fused subtree-expansion kernel KExpand<D, Emitter>
// (ExpandSeeds cc:289-372 + HashExpandedSeeds cc:523-547 + the correction loop
// of EvaluateUntil h:836-862) and its leaf emitters.  Included by the
// k_expand_*.hip translation units, each instantiating a few emitters.
#pragma once

// At 6 waves/SIMD the compiler's own interleaving of the table reads beats
// forcing a round's reads into one group (fewer live VGPRs).
#ifndef DPF_AES_SCHED
#define DPF_AES_SCHED 0
#endif
#include "aes_device.h"

#ifndef DPF_EXPAND_EXTRA_DEPTHS
#define DPF_EXPAND_EXTRA_DEPTHS 0  // KExpand<3> for A/B builds
#endif

#ifndef DPF_EXPAND_MAX_GRID
#define DPF_EXPAND_MAX_GRID (1 << 24)
#endif

// Leaves a lane keeps in registers before storing them as one contiguous
// burst (0: every leaf is stored as it is produced).  A lane's leaves are
// consecutive in the output, so 8 x 16 B fill a whole 128-byte line at once
// instead of leaving it partly written in L2 across 8 leaves of compute.
// The 32 staging VGPRs need the 4-wave/SIMD register budget, so the staged
// emitters launch 512-thread blocks (2 per CU, one 64 KiB table each).
// Measured on MI355X, c5 KExpand<8, EmitU32ModN64>: 178.8 ms unstaged at 6
// waves/SIMD (19 VGPRs spilled to scratch), 181.2 ms unstaged at 4, 164.6 ms
// staged at 4 (no spills), 171.3 ms staged at 5.
#ifndef DPF_STAGE_LEAVES
#define DPF_STAGE_LEAVES 8
#endif
#ifndef DPF_STAGED_BLOCK
#define DPF_STAGED_BLOCK 512
#define DPF_STAGED_WAVES 4
#endif

namespace dpf_amd {

template <int BN>
struct EmitGeneric {
  static constexpr int kBN = BN;
  static constexpr bool kCanStage = false;
  static constexpr bool kCanBatch = false;
  __device__ static void Emit(const ExpandCtx& E, const uint32_t (&h)[BN][4], uint32_t t,
                              int64_t g) {
    const VtDev& vt = E.vt;
    if (g < E.a.leaf_begin || g >= E.a.leaf_end) return;
    u128 W[BN];
#pragma unroll
    for (int j = 0; j < BN; ++j) W[j] = ToU128(h[j]);
    char* base = E.a.out + (g - E.a.leaf_begin) * (int64_t)vt.cepb * vt.stride;
    const int stride = vt.stride;
    EmitLeaf<BN>(vt, W, t != 0, vt.party, vt.corr, 0, vt.cepb,
                 [base, stride](int e) { return base + (int64_t)e * stride; });
  }
};

// Lane-wise (SWAR) arithmetic on a 16-byte block of B-byte integers.
template <int B>
__device__ __forceinline__ void SwarAdd(uint32_t (&a)[4], const uint32_t (&b)[4]) {
  if constexpr (B == 16) {
    FromU128(ToU128(a) + ToU128(b), a);
  } else if constexpr (B == 8) {
#pragma unroll
    for (int i = 0; i < 4; i += 2) {
      uint64_t x = ((uint64_t)a[i + 1] << 32 | a[i]) + ((uint64_t)b[i + 1] << 32 | b[i]);
      a[i] = (uint32_t)x;
      a[i + 1] = (uint32_t)(x >> 32);
    }
  } else if constexpr (B == 4) {
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] += b[i];
  } else {
    constexpr uint32_t H = (B == 2) ? 0x80008000u : 0x80808080u;
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = ((a[i] & ~H) + (b[i] & ~H)) ^ ((a[i] ^ b[i]) & H);
  }
}

template <int B>
__device__ __forceinline__ void SwarNeg(uint32_t (&a)[4]) {
  if constexpr (B == 16) {
    FromU128((u128)0 - ToU128(a), a);
  } else if constexpr (B == 8) {
#pragma unroll
    for (int i = 0; i < 4; i += 2) {
      uint64_t x = 0 - ((uint64_t)a[i + 1] << 32 | a[i]);
      a[i] = (uint32_t)x;
      a[i + 1] = (uint32_t)(x >> 32);
    }
  } else if constexpr (B == 4) {
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = 0u - a[i];
  } else {
    constexpr uint32_t one = (B == 2) ? 0x00010001u : 0x01010101u;
    uint32_t o[4] = {one, one, one, one};
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = ~a[i];
    SwarAdd<B>(a, o);
  }
}

// T is a single directly-convertible B-byte integer or XorWrapper
// (uint8..uint128, XorWrapper<uint8..uint128>): the elements of a leaf are the
// consecutive B-byte slices of the hashed block (vth:586-598).
// One 16-byte leaf output in host layout (the packed emitters' common store).
__device__ __forceinline__ void StoreLeaf16(const ExpandCtx& E, const uint4& v, int64_t g) {
  if (g < E.a.leaf_begin || g >= E.a.leaf_end) return;
  uint4* dst = reinterpret_cast<uint4*>(E.a.out) + (g - E.a.leaf_begin);
#if DPF_EXPERIMENT_STORE == 1  // measurement only: almost no stores
  if (v.z == 0x9e3779b9u) *dst = v;
#elif DPF_EXPERIMENT_STORE == 2  // nontemporal stores
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  u32x4 vv = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(vv, reinterpret_cast<u32x4*>(dst));
#else
  *dst = v;
#endif
}

template <int B>
struct EmitDirect {
  static constexpr int kBN = 1;
  static constexpr bool kCanStage = true;  // when Packed(vt)
  // Whole 16-byte blocks per leaf (every element of the block is returned).
  __device__ static bool Packed(const VtDev& vt) { return vt.cepb * B == 16; }
  static constexpr bool kCanBatch = true;  // per-key corrections (ExpandCtx::per_key)
  __device__ static uint4 Value(const ExpandCtx& E, const uint32_t (&h)[1][4], uint32_t t) {
    const VtDev& vt = E.vt;
    uint32_t w[4], c[4];
    const uint32_t m = 0u - t;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      w[i] = h[0][i];
      c[i] = (E.per_key ? E.kcorr[i] : (uint32_t)(vt.corr_packed >> (32 * i))) & m;
    }
    const int party = E.per_key ? E.kparty : vt.party;
    if (vt.sc[0].kind == DPF_AMD_KIND_XOR_WRAPPER) {
#pragma unroll
      for (int i = 0; i < 4; ++i) w[i] ^= c[i];
    } else {
      SwarAdd<B>(w, c);
      if (party == 1) SwarNeg<B>(w);
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
  __device__ static void Emit(const ExpandCtx& E, const uint32_t (&h)[1][4], uint32_t t,
                              int64_t g) {
    const VtDev& vt = E.vt;
    const uint4 w = Value(E, h, t);
    if (Packed(vt)) {
      StoreLeaf16(E, w, g);
      return;
    }
    if (g < E.a.leaf_begin || g >= E.a.leaf_end) return;
    char* dst = E.a.out + (g - E.a.leaf_begin) * (int64_t)vt.cepb * B;
    const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
    const u128 v = ToU128(ww);
    for (int e = 0; e < vt.cepb; ++e) StoreScalar(dst + e * B, B, v >> (8 * B * e));
  }
};

// T = Tuple<uint32_t, IntModN<uint64_t, m>> with m = 2^64 - c, c < 2^56
// (the c5 benchmark type).  Sampling path of vth:230-251, 303-328, 447-460:
// element 0 = low 32 bits of block 0; block := (block & ~0xffffffff) |
// bytes[16..20); element 1 = block mod m.
struct EmitU32ModN64 {
  static constexpr int kBN = 2;
  static constexpr bool kCanStage = true;  // when Packed(vt)
  static constexpr bool kCanBatch = false;
  // libstdc++ tuple layout: u64 at 0, u32 at 8, stride 16.
  __device__ static bool Packed(const VtDev& vt) {
    return vt.sc[0].out_off == 8 && vt.sc[1].out_off == 0 && vt.stride == 16;
  }
  __device__ static void Elements(const ExpandCtx& E, const uint32_t (&h)[2][4], uint32_t t,
                                  uint32_t& v0, uint64_t& v1) {
    const VtDev& vt = E.vt;
    v0 = h[0][0];
    const uint64_t lo = (uint64_t)h[0][1] << 32 | h[1][0];
    const uint64_t hi = (uint64_t)h[0][3] << 32 | h[0][2];
    const uint64_t c = (uint64_t)vt.sc[1].fold_c;
    const uint64_t mod = (uint64_t)vt.sc[1].mod;
    // x = hi * 2^64 + lo = hi * c + lo (mod m); fold until it fits 64 bits.
    uint64_t xlo = lo, xhi = hi;
    while (xhi != 0) {
      const uint64_t plo = xhi * c, phi = __umul64hi(xhi, c);
      xlo = plo + xlo;
      xhi = phi + (xlo < plo ? 1 : 0);
    }
    v1 = xlo >= mod ? xlo - mod : xlo;
    if (t) {
      v0 += (uint32_t)vt.corr[0];
      const uint64_t c1 = (uint64_t)vt.corr[1];
      const uint64_t x = mod - c1;
      v1 = v1 >= x ? v1 - x : v1 + c1;
    }
    if (vt.party == 1) {
      v0 = 0u - v0;
      v1 = v1 ? mod - v1 : 0;
    }
  }
  __device__ static uint4 Value(const ExpandCtx& E, const uint32_t (&h)[2][4], uint32_t t) {
    uint32_t v0;
    uint64_t v1;
    Elements(E, h, t, v0, v1);
    return make_uint4((uint32_t)v1, (uint32_t)(v1 >> 32), v0, 0u);
  }
  __device__ static void Emit(const ExpandCtx& E, const uint32_t (&h)[2][4], uint32_t t,
                              int64_t g) {
    const VtDev& vt = E.vt;
    if (Packed(vt)) {
      StoreLeaf16(E, Value(E, h, t), g);
      return;
    }
    if (g < E.a.leaf_begin || g >= E.a.leaf_end) return;
    uint32_t v0;
    uint64_t v1;
    Elements(E, h, t, v0, v1);
    char* dst = E.a.out + (g - E.a.leaf_begin) * (int64_t)vt.stride;
    *reinterpret_cast<uint32_t*>(dst + vt.sc[0].out_off) = v0;
    *reinterpret_cast<uint64_t*>(dst + vt.sc[1].out_off) = v1;
  }
};

// ----------------------------------------------------------------------------
// Fused subtree expansion kernel: each thread walks from its root to the root
// of a 2^D-leaf subtree (one AES per level, the path child only), then expands
// it depth-first in registers (right children kept per level, their control
// bit packed into the always-zero LSB of the seed), hashes and emits every
// leaf.  The DFS position j is wave-uniform (an SGPR); a lane's leaf index is
// (chunk << D) + j.
// ----------------------------------------------------------------------------

template <class Em>
constexpr bool kStagedEm = DPF_STAGE_LEAVES > 0 && Em::kCanStage;
template <class Em>
constexpr int kBlockOf = kStagedEm<Em> ? DPF_STAGED_BLOCK : kExpandBlock;
template <class Em>
constexpr int kWavesOf = kStagedEm<Em> ? DPF_STAGED_WAVES : kExpandWaves;

struct LeafStage {
  uint4 v[DPF_STAGE_LEAVES > 0 ? DPF_STAGE_LEAVES : 1];
};

template <class Em, int D>
constexpr bool kStaged = kStagedEm<Em> && (1 << D) >= DPF_STAGE_LEAVES;

// Leaf j of the lane's subtree (j wave-uniform): staged when the emitter
// writes packed 16-byte leaves, flushed as one burst per DPF_STAGE_LEAVES.
// Progress-ordered wave priority.  The sequencer favours older waves, so
// within a round of resident blocks the oldest waves run ahead and finish
// first, and the last ones run alone at an occupancy too low to keep the
// LDS busy (tools/expand_trace.py: one round's waves ended between 78 and
// 162 us, four per SIMD one after another).  A wave starts at priority 3 and
// steps down one level per quarter of its subtree's leaves, so waves that
// are behind are served first and a round's waves finish together (122-150
// us).  Measured: one rank's c5 slice at N = 8 19.77-19.99 -> 19.28-19.36
// ms, the whole c5 domain 153.9-154.1 -> 152.7-153.1 ms, c3's launch shape
// -5 % (profiles/c5_slice_prio_r06/, ab_expand_prio_r06t/, r06u/).
// DPF_EXPAND_PRIO=0 turns it off, 2 steps at 3/4, 7/8 and 15/16 instead.
#ifndef DPF_EXPAND_PRIO
#define DPF_EXPAND_PRIO 1
#endif
template <int D>
__device__ __forceinline__ void ProgressPrio(int j) {
  if constexpr (DPF_EXPAND_PRIO == 2 && D >= 2) {
    // geometric: priority 3 up to 3/4 of the leaves, 2 to 7/8, 1 to 15/16
    // (D = 2: 3/4 only), so the final spread is at most 1/16 of the work
    const int done = j + 1;
    constexpr int n = 1 << D;
    if (done == n - n / 4)
      __builtin_amdgcn_s_setprio(2);
    else if (D >= 3 && done == n - n / 8)
      __builtin_amdgcn_s_setprio(1);
    else if (D >= 4 && done == n - n / 16)
      __builtin_amdgcn_s_setprio(0);
  } else if constexpr (DPF_EXPAND_PRIO == 1 && D >= 2) {
    const int done = j + 1;  // leaves emitted (wave-uniform)
    if ((done & ((1 << (D - 2)) - 1)) == 0) {
      const int q = done >> (D - 2);  // quarters done, 1..4
      if (q == 1)
        __builtin_amdgcn_s_setprio(2);
      else if (q == 2)
        __builtin_amdgcn_s_setprio(1);
      else if (q == 3)
        __builtin_amdgcn_s_setprio(0);
    }
  }
}

template <int D, class Em, int BN>
__device__ __forceinline__ void EmitStagedLeaf(const ExpandCtx& E, LeafStage& S,
                                         const uint32_t (&h)[BN][4], uint32_t t,
                                         int64_t chunk, int j) {
  if constexpr (kStaged<Em, D>) {
    if (Em::Packed(E.vt)) {
      constexpr int N = DPF_STAGE_LEAVES;
      const uint4 v = Em::Value(E, h, t);
      const int k = j & (N - 1);
#pragma unroll
      for (int i = 0; i < N; ++i)
        if (i == k) S.v[i] = v;
      if (k == N - 1) {
        const int64_t g0 = (chunk << D) + j - (N - 1);
        if (g0 >= E.a.leaf_begin && g0 + N <= E.a.leaf_end) {
          uint4* dst = reinterpret_cast<uint4*>(E.a.out) + (g0 - E.a.leaf_begin);
#pragma unroll
          for (int i = 0; i < N; ++i) dst[i] = S.v[i];
        } else {
#pragma unroll
          for (int i = 0; i < N; ++i) StoreLeaf16(E, S.v[i], g0 + i);
        }
      }
      ProgressPrio<D>(j);
      return;
    }
  }
  Em::Emit(E, h, t, (chunk << D) + j);
  ProgressPrio<D>(j);
}

template <int DEPTH, int D, class Em>
__device__ __forceinline__ void Dfs(const ExpandCtx& E, LeafStage& S, const uint32_t (&x)[4],
                                    uint32_t t, int level, int64_t chunk, int j) {
  constexpr int BN = Em::kBN;
  if constexpr (DEPTH == 0) {
    uint32_t xs[1][4] = {{x[0], x[1], x[2], x[3]}};
    uint32_t h[1][BN][4];
    // For D > 0 the seed comes out of Expand2 with its LSB cleared.
    HashWords<1, BN, (D > 0)>(xs, h, E.L);
    EmitStagedLeaf<D, Em, BN>(E, S, h[0], t, chunk, j);
  } else {
    const Cw cw = LoadCw(E.a.cw_seed, E.a.ccl, E.a.ccr, E.cw0 + level);
    uint32_t l[4], r[4], tl, tr;
    Expand2(x, t, cw, E.L, l, tl, r, tr);
    if constexpr (DEPTH == 1 && BN == 1) {
      uint32_t xs[2][4] = {{l[0], l[1], l[2], l[3]}, {r[0], r[1], r[2], r[3]}};
      uint32_t h[2][1][4];
      HashWords<2, 1>(xs, h, E.L);
      EmitStagedLeaf<D, Em, 1>(E, S, h[0], tl, chunk, 2 * j);
      EmitStagedLeaf<D, Em, 1>(E, S, h[1], tr, chunk, 2 * j + 1);
    } else {
      // Only the right child stays live across the left recursion (its
      // control bit packed into its seed's LSB); the left child is consumed
      // by the first iteration.
      r[0] |= tr;
      uint32_t y[4] = {l[0], l[1], l[2], l[3]};
      uint32_t ty = tl;
#pragma unroll 1
      for (int b = 0; b < 2; ++b) {
        Dfs<DEPTH - 1, D, Em>(E, S, y, ty, level + 1, chunk, 2 * j + b);
#pragma unroll
        for (int c = 0; c < 4; ++c) y[c] = r[c];
        ty = y[0] & 1u;
        y[0] &= ~1u;
      }
    }
  }
}

// Batched keys (kBatched, ExpandArgs::batched): lane i's chunk id maps to
// key id / (chunk_end - chunk_begin) with that key's root, correction words,
// value correction and party; leaf ranges and outputs are per key.
// Per-wave timestamps of KExpand (diagnostic builds only: tools/expand_trace.py
// builds one translation unit with DPF_EXPAND_TRACE=1): per wave, lane 0's
// s_memrealtime (100 MHz) at entry, after the tables, after the walk and at
// the end (slots 0-3), s_memtime (shader clock) at entry and end (4-5), and
// the HW_ID / XCC_ID registers (6-7).
#if DPF_EXPAND_TRACE
__device__ uint64_t g_expand_trace[16384 * 8];
extern "C" __attribute__((visibility("default"))) int dpf_amd_debug_expand_trace(void* host,
                                                                                 int64_t bytes) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_expand_trace), (size_t)bytes, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}
#define DPF_EXP_MARK(i, v)                                                          \
  do {                                                                              \
    const int w_ = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);             \
    if ((threadIdx.x & 63) == 0 && w_ < 16384) g_expand_trace[w_ * 8 + (i)] = (v); \
  } while (0)
#else
#define DPF_EXP_MARK(i, v) \
  do {                     \
  } while (0)
#endif

template <int D, class Em, bool kBatched = false>
__global__ __launch_bounds__(kBlockOf<Em>, kWavesOf<Em>) void KExpand(ExpandArgs a, VtDev vt) {
  __shared__ uint32_t tab[kTabWords];
  DPF_EXP_MARK(0, __builtin_amdgcn_s_memrealtime());
  DPF_EXP_MARK(4, __builtin_amdgcn_s_memtime());
  DPF_EXP_MARK(6, (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4));
  DPF_EXP_MARK(7, (uint64_t)__builtin_amdgcn_s_getreg((3 << 11) | 20));
  FillTables(tab);
  __syncthreads();
  DPF_EXP_MARK(1, __builtin_amdgcn_s_memrealtime());
  const Lds L = MakeLds(tab);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t cpk = a.chunk_end - a.chunk_begin;
  const int64_t total = kBatched ? cpk * a.num_keys : cpk;
  // Every lane runs the same number of iterations (uniform trip count), so
  // the per-level wave votes below see all lanes; lanes past the end idle.
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x; base < total; base += stride) {
    if (DPF_EXPAND_PRIO) __builtin_amdgcn_s_setprio(3);
    const int64_t id = base + threadIdx.x;
    const bool live = id < total;
    const int64_t cid = live ? id : total - 1;
    const int64_t key = kBatched ? cid / cpk : 0;
    const int64_t c = a.chunk_begin + (kBatched ? cid - key * cpk : cid);
    const int64_t root = kBatched ? key : (c >> a.walk) - a.root_base;
    // first correction word of the walk: [key][level] when batched, else the
    // level of the precomputed roots (0: the key's root)
    const int64_t cw0 = kBatched ? key * a.num_levels : a.root_level;
    const uint64_t path = (uint64_t)c & ((a.walk >= 63) ? ~0ull : ((1ull << a.walk) - 1));
    uint4 s = a.root_seeds[root];
    uint32_t x[4] = {s.x, s.y, s.z, s.w};
    uint32_t t;
    if (!kBatched && a.root_cb == nullptr) {  // packed node: control bit in the LSB
      t = x[0] & 1u;
      x[0] &= ~1u;
    } else {
      t = a.root_cb[root];
    }
    for (int i = 0; i < a.walk; ++i) {
      const uint32_t bit = (uint32_t)(path >> (a.walk - 1 - i)) & 1u;
      const Cw cw = LoadCw(a.cw_seed, a.ccl, a.ccr, cw0 + i);
      // The upper path bits are shared by the whole wave: one AES with the
      // key picked by a scalar select.  Lanes that disagree compute both
      // children with the uniform keys and keep the path child.
      if (__ballot(bit) == 0 || __ballot(bit ^ 1u) == 0) {
        const uint32_t ubit = __builtin_amdgcn_readfirstlane(bit);
        WalkStep(x, t, ubit, cw, DpfSelect{{}, ubit != 0}, L);
      } else if (DPF_LANE_WALK) {
        // Divergent bits: one AES, round keys selected per lane (VALU
        // v_cndmask per key word, no extra LDS lookups).
        WalkStep(x, t, bit, cw, DpfMasked<1>{{0u - bit}}, L);
      } else {
        uint32_t l[4], r[4], tl, tr;
        Expand2(x, t, cw, L, l, tl, r, tr);
#pragma unroll
        for (int c = 0; c < 4; ++c) x[c] = bit ? r[c] : l[c];
        t = bit ? tr : tl;
      }
    }
    DPF_EXP_MARK(2, __builtin_amdgcn_s_memrealtime());
    ExpandArgs ak = a;
    ExpandCtx E{ak, vt, L};
    if constexpr (kBatched) {
      ak.out += key * a.key_out_stride;
      const uint4 kc = a.key_corr[key];
      E.per_key = true;
      E.kcorr[0] = kc.x;
      E.kcorr[1] = kc.y;
      E.kcorr[2] = kc.z;
      E.kcorr[3] = kc.w;
      E.kparty = a.key_party[key];
      E.cw0 = cw0;
    }
    LeafStage S;
    if (live) Dfs<D, D, Em>(E, S, x, t, kBatched ? a.walk : a.root_level + a.walk, c, 0);
  }
  DPF_EXP_MARK(3, __builtin_amdgcn_s_memrealtime());
  DPF_EXP_MARK(5, __builtin_amdgcn_s_memtime());
}

template <int D, class Em>
int LaunchExpand(int, hipStream_t st, const ExpandArgs& a, const VtDev& vt) {
  // One subtree per thread, many more blocks than resident slots: blocks
  // finish at different times (per-CU clocks differ) and the dispatcher
  // back-fills.  c5: 2^24 subtrees / 768 = 21845 blocks -> 166.8 ms, vs
  // 173.8 ms capped at 2730 blocks and 180.5 ms at one resident round.
  constexpr int block = kBlockOf<Em>;
  const int64_t chunks = (a.chunk_end - a.chunk_begin) * (a.batched ? a.num_keys : 1);
  const int grid = (int)std::max<int64_t>(
      1, std::min<int64_t>((chunks + block - 1) / block, DPF_EXPAND_MAX_GRID));
  if (a.batched) {
    if constexpr (Em::kCanBatch) {
      hipLaunchKernelGGL((KExpand<D, Em, true>), dim3(grid), dim3(block), 0, st, a, vt);
    } else {
      return SetError(DPF_AMD_INTERNAL, "batched expansion needs a directly convertible type");
    }
  } else {
    hipLaunchKernelGGL((KExpand<D, Em, false>), dim3(grid), dim3(block), 0, st, a, vt);
  }
  return LaunchCheck("expand kernel launch");
}

// ----------------------------------------------------------------------------
// KExpandCoop<E, Em, kBatched>: cooperative expansion for launches below
// 2^25 tree leaves and for batches of keys (the selection vectors of a PIR
// request).  KExpand gives every thread its own walk from the root, which
// small launches cannot amortise (a 2^19-leaf launch at D = 2: 27 AES per 4
// leaves against 12, and a 17-AES chain per thread).  Here a block owns a
// 2^(10+E)-leaf subtree and computes every tree node of it once:
//   1. waves 0-3, as 64 quads of lanes sharing one AES state (lane c holds
//      column c), walk from the root to the block root (block-uniform path
//      bits) and on to 64 sub-roots six levels below, quad q to sub-root q;
//   2. four breadth-first levels through LDS, one child per thread (a walk
//      step with the key of the child's side): 64 -> 128 -> ... -> 1024;
//   3. each thread hashes its node (E = 0) or expands it once more and
//      hashes both children (E = 1), converts, corrects and stores —
//      consecutive threads write consecutive leaves.
// Per 2^10 leaves (E = 0, BN = 1): (s + 6) + 30 + 16 wave-AES for 48
// algorithmic, s = tree depth of the block root.
// ----------------------------------------------------------------------------

#ifndef DPF_COOP_BLOCK
#define DPF_COOP_BLOCK 1024
#endif
#ifndef DPF_COOP_WAVES
#define DPF_COOP_WAVES 8  // 2 blocks per CU (72 KiB LDS each)
#endif
constexpr int kCoopBlock = DPF_COOP_BLOCK;
#ifndef DPF_COOP_QUAD_BFS
// breadth-first levels run as quad steps (0-3; 2: c1 span 38.9 -> 36.5 us;
// 3: the 512-child level as quads expanding both children of a parent)
#define DPF_COOP_QUAD_BFS 3
#endif
static_assert(DPF_COOP_QUAD_BFS >= 0 && DPF_COOP_QUAD_BFS <= 3, "quad BFS levels: 0-3");

// Phase timestamps of KExpandCoop (diagnostic builds only: tools/coop_trace.py
// builds one translation unit with DPF_COOP_TRACE=1): per block, thread 0's
// s_memrealtime (100 MHz) at entry, after the tables, after the walk, after
// the BFS and at the end (slots 0-4), after each quad BFS level (5-7).
#if DPF_COOP_TRACE
__device__ uint64_t g_coop_trace[4096 * 8];
__device__ uint64_t g_coop_clock[4096 * 8];  // s_memtime (shader clock) at the same marks
#define DPF_COOP_MARK(i)                                                      \
  do {                                                                        \
    if (DPF_COOP_TRACE_SYNC) __syncthreads();                                 \
    if (threadIdx.x == 0 && blockIdx.x < 4096) {                              \
      g_coop_trace[blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memrealtime();  \
      g_coop_clock[blockIdx.x * 8 + (i)] = __builtin_amdgcn_s_memtime();      \
    }                                                                         \
  } while (0)
extern "C" __attribute__((visibility("default"))) int dpf_amd_debug_coop_trace(void* host,
                                                                               int64_t bytes) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_coop_trace), (size_t)bytes, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}
extern "C" __attribute__((visibility("default"))) int dpf_amd_debug_coop_clock(void* host,
                                                                               int64_t bytes) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_coop_clock), (size_t)bytes, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}
#else
#define DPF_COOP_MARK(i) \
  do {                   \
  } while (0)
#endif
#ifndef DPF_COOP_TRACE_SYNC
#define DPF_COOP_TRACE_SYNC 1
#endif
static_assert(kCoopBlock == 1024, "the BFS levels assume 1024 threads (64 -> 1024 nodes)");
constexpr int kCoopLog = 10;  // log2 nodes after the BFS

// Tree nodes instead of leaves: KExpandCoop<0, EmitNodes> stores node g of its
// last level as one packed 16-byte word (control bit in the seed's LSB) at
// out[g - leaf_begin] — the roots stage of a large expansion
// (dpf_amd_expand_and_correct), which KExpand then starts from.
struct EmitNodes {
  static constexpr int kBN = 1;
  static constexpr bool kCanStage = false;
  static constexpr bool kCanBatch = false;
};
template <class Em>
inline constexpr bool kNodesEm = false;
template <>
inline constexpr bool kNodesEm<EmitNodes> = true;

template <int E, class Em, bool kBatched>
__global__ __launch_bounds__(kCoopBlock, DPF_COOP_WAVES) void KExpandCoop(ExpandArgs a,
                                                                          VtDev vt) {
  __shared__ uint32_t tab[kTabWords];
  __shared__ uint4 nodes[kCoopBlock / 2];
  constexpr int BN = Em::kBN;
  constexpr int K = kCoopLog + E;  // log2 tree leaves per block
  DPF_COOP_MARK(0);
  FillTables(tab);
  __syncthreads();
  DPF_COOP_MARK(1);
  const Lds L = MakeLds(tab);
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int64_t cpk = a.chunk_end - a.chunk_begin;  // blocks per key
  const int64_t key = kBatched ? (int64_t)blockIdx.x / cpk : 0;
  const int64_t chunk = a.chunk_begin + (kBatched ? (int64_t)blockIdx.x % cpk : blockIdx.x);
  const int s = a.walk;  // tree depth of the block root (below its root seed)
  const int64_t root = kBatched ? key : chunk >> s;
  const uint64_t path = (uint64_t)chunk & ((s >= 63) ? ~0ull : ((1ull << s) - 1));
  const int64_t cw0 = kBatched ? key * a.num_levels : 0;
  // 1. root -> block root -> 64 sub-roots: waves 0-3 as 64 quads (four lanes
  // per state, lane c holding column c: a lone chain's AES at a quarter of
  // the lookups per lane), quad q walking to sub-root q; the walk to the
  // block root is the same for every quad (block-uniform path bits).
  if (wave < 4) {
    const int c = lane & 3;
    const int q = wave * 16 + (lane >> 2);
    const QuadKey kl = MakeQuadKey<0>(c);
    const QuadDiff kd = MakeQuadDiff(c);
    const uint32_t* cw_words = reinterpret_cast<const uint32_t*>(a.cw_seed);
    uint32_t x = reinterpret_cast<const uint32_t*>(a.root_seeds)[root * 4 + c];
    uint32_t t = a.root_cb[root];
#pragma unroll 1
    for (int i = 0; i < s; ++i) {
      const uint32_t bit = (uint32_t)(path >> (s - 1 - i)) & 1u;  // block-uniform
      const int64_t ci = cw0 + i;
      QuadWalkStep(x, t, bit, cw_words[ci * 4 + c], a.ccl[ci], a.ccr[ci], c, kl, kd, L);
    }
#pragma unroll 1
    for (int i = 0; i < 6; ++i) {
      const uint32_t bit = ((uint32_t)q >> (5 - i)) & 1u;
      const int64_t ci = cw0 + s + i;
      QuadWalkStep(x, t, bit, cw_words[ci * 4 + c], a.ccl[ci], a.ccr[ci], c, kl, kd, L);
    }
    reinterpret_cast<uint32_t*>(nodes)[q * 4 + c] = c == 0 ? (x | t) : x;
  }
  __syncthreads();
  DPF_COOP_MARK(2);
  // 2. breadth-first: level j has 128 << j children, child c of parent c / 2.
  // The first DPF_COOP_QUAD_BFS levels (128 and 256 children: half and all
  // of the block as quads) run as quad steps like the walk — a lone lane-AES
  // at 2-4 waves per CU is latency-bound (~2.9 us per level measured,
  // tools/coop_trace.py; the four levels 11.7 -> 9.7 us with two quad levels,
  // profiles/coop_quad_bfs_r03r.log); the rest one child per thread.
#if DPF_COOP_QUAD_BFS > 0
  {
    const int c = lane & 3;
    const int qd = tid >> 2;
    const QuadKey kl = MakeQuadKey<0>(c);
    const QuadDiff kd = MakeQuadDiff(c);
    const uint32_t* cw_words = reinterpret_cast<const uint32_t*>(a.cw_seed);
    uint32_t* nw = reinterpret_cast<uint32_t*>(nodes);
#pragma unroll
    for (int j = 0; j < (DPF_COOP_QUAD_BFS < 2 ? DPF_COOP_QUAD_BFS : 2); ++j) {
      const bool active = wave < (8 << j);  // 128 << j quads, 16 per wave
      uint32_t xq = 0u, tq = 0u;
      if (active) {
        const uint32_t w = nw[(qd >> 1) * 4 + c];
        tq = QuadPerm<kQuadBcast<0>>(w) & 1u;
        xq = c == 0 ? (w & ~1u) : w;
        const int64_t ci = cw0 + s + 6 + j;
        QuadWalkStep(xq, tq, (uint32_t)qd & 1u, cw_words[ci * 4 + c], a.ccl[ci], a.ccr[ci], c,
                     kl, kd, L);
      }
      __syncthreads();  // every parent of this level has been read
      if (active) nw[qd * 4 + c] = c == 0 ? (xq | tq) : xq;
      __syncthreads();
      DPF_COOP_MARK(5 + j);
    }
    if constexpr (E == -2) {
      static_assert(DPF_COOP_QUAD_BFS >= 2, "E = -2 ends on the second quad level");
      // 256 leaves per block (launches too small to give every CU a
      // 1024-leaf block): the 256-node level is the last; node qd is hashed
      // on its quad with the value key (HashWords' blocks H_V(seed + j) as
      // quad rounds, the 128-bit seed + j formed from the broadcast columns)
      // and the quad's lane 0 converts, corrects and stores it.
      static_assert(!kNodesEm<Em>, "nodes are stored from the 1024-node level");
      const uint32_t w = nw[qd * 4 + c];
      const uint32_t tq = QuadPerm<kQuadBcast<0>>(w) & 1u;
      const uint32_t xq = c == 0 ? (w & ~1u) : w;
      const QuadRk kvr = MakeQuadRk<2>(c);
      uint32_t h[BN][4];
#pragma unroll
      for (int j = 0; j < BN; ++j) {
        uint32_t in = xq;
        if (j > 0) {
          const u128 v = ((u128)QuadPerm<kQuadBcast<0>>(xq) |
                          ((u128)QuadPerm<kQuadBcast<1>>(xq) << 32) |
                          ((u128)QuadPerm<kQuadBcast<2>>(xq) << 64) |
                          ((u128)QuadPerm<kQuadBcast<3>>(xq) << 96)) +
                         (u128)j;
          in = (uint32_t)(v >> (32 * c));
        }
        const uint32_t sg = SigmaQuad(in, c);
        const uint32_t hv = AesQuadRk<false>(sg, kvr, L) ^ sg;
        h[j][0] = QuadPerm<kQuadBcast<0>>(hv);
        h[j][1] = QuadPerm<kQuadBcast<1>>(hv);
        h[j][2] = QuadPerm<kQuadBcast<2>>(hv);
        h[j][3] = QuadPerm<kQuadBcast<3>>(hv);
      }
      ExpandArgs ak = a;
      if constexpr (kBatched) ak.out += key * a.key_out_stride;
      ExpandCtx Ec{ak, vt, L};
      if constexpr (kBatched) {
        const uint4 kc = a.key_corr[key];
        Ec.per_key = true;
        Ec.kcorr[0] = kc.x;
        Ec.kcorr[1] = kc.y;
        Ec.kcorr[2] = kc.z;
        Ec.kcorr[3] = kc.w;
        Ec.kparty = a.key_party[key];
      }
      if (c == 0) Em::Emit(Ec, h, tq, (chunk << K) + qd);
      DPF_COOP_MARK(4);
      return;
    }
#if DPF_COOP_QUAD_BFS > 2
    {
      // 512 children: quad qd (all 256 of them) expands parent qd into
      // children 2qd and 2qd + 1 — two independent quad chains per lane
      // instead of one lane-AES per child (latency-bound at 8 waves per CU)
      const uint32_t w = nw[qd * 4 + c];
      const uint32_t tp = QuadPerm<kQuadBcast<0>>(w) & 1u;
      uint32_t x0 = c == 0 ? (w & ~1u) : w, x1 = x0, t0 = tp, t1 = tp;
      const int64_t ci = cw0 + s + 6 + 2;
      const uint32_t cwc = cw_words[ci * 4 + c];
      const uint32_t cl = a.ccl[ci], cr = a.ccr[ci];
      QuadWalkStep(x0, t0, 0u, cwc, cl, cr, c, kl, kd, L);
      QuadWalkStep(x1, t1, 1u, cwc, cl, cr, c, kl, kd, L);
      __syncthreads();  // every parent has been read
      nw[(2 * qd) * 4 + c] = c == 0 ? (x0 | t0) : x0;
      nw[(2 * qd + 1) * 4 + c] = c == 0 ? (x1 | t1) : x1;
      __syncthreads();
      DPF_COOP_MARK(7);
    }
#endif
  }
#endif
  uint32_t x[4] = {0u, 0u, 0u, 0u}, t = 0;
#pragma unroll
  for (int j = DPF_COOP_QUAD_BFS; j < 4; ++j) {
    const bool active = wave < (2 << j);  // wave-uniform
    if (active) {
      const uint4 p = nodes[tid >> 1];
      x[0] = p.x & ~1u;
      x[1] = p.y;
      x[2] = p.z;
      x[3] = p.w;
      t = p.x & 1u;
      const uint32_t bit = (uint32_t)tid & 1u;
      const Cw cw = LoadCw(a.cw_seed, a.ccl, a.ccr, cw0 + s + 6 + j);
      WalkStep(x, t, bit, cw, DpfMasked<1>{{0u - bit}}, L);
    }
    if (j < 3) {
      __syncthreads();  // every parent of this level has been read
      if (active) nodes[tid] = make_uint4(x[0] | t, x[1], x[2], x[3]);
      __syncthreads();
    }
  }
  DPF_COOP_MARK(3);
  // 3. leaves: hash, convert, correct, store
  ExpandArgs ak = a;
  if constexpr (kBatched) ak.out += key * a.key_out_stride;
  ExpandCtx Ec{ak, vt, L};
  if constexpr (kBatched) {
    const uint4 c = a.key_corr[key];
    Ec.per_key = true;
    Ec.kcorr[0] = c.x;
    Ec.kcorr[1] = c.y;
    Ec.kcorr[2] = c.z;
    Ec.kcorr[3] = c.w;
    Ec.kparty = a.key_party[key];
  }
  const int64_t g0 = chunk << K;  // first tree leaf of the block (per key if batched)
  if constexpr (kNodesEm<Em>) {
    static_assert(E == 0 && !kBatched, "nodes are stored from the 1024-node level");
    const int64_t g = g0 + tid;
    if (g >= a.leaf_begin && g < a.leaf_end)
      reinterpret_cast<uint4*>(a.out)[g - a.leaf_begin] =
          make_uint4((x[0] & ~1u) | t, x[1], x[2], x[3]);
  } else if constexpr (E == 0) {
    uint32_t xs[1][4] = {{x[0], x[1], x[2], x[3]}};
    uint32_t h[1][BN][4];
    HashWords<1, BN, true>(xs, h, L);
    Em::Emit(Ec, h[0], t, g0 + tid);
  } else {
    const Cw cw = LoadCw(a.cw_seed, a.ccl, a.ccr, cw0 + s + 10);
    uint32_t l[4], r[4], tl, tr;
    Expand2(x, t, cw, L, l, tl, r, tr);
    if constexpr (BN == 1) {
      uint32_t xs[2][4] = {{l[0], l[1], l[2], l[3]}, {r[0], r[1], r[2], r[3]}};
      uint32_t h[2][1][4];
      HashWords<2, 1, true>(xs, h, L);
      Em::Emit(Ec, h[0], tl, g0 + 2 * tid);
      Em::Emit(Ec, h[1], tr, g0 + 2 * tid + 1);
    } else {
      uint32_t xl[1][4] = {{l[0], l[1], l[2], l[3]}};
      uint32_t h[1][BN][4];
      HashWords<1, BN, true>(xl, h, L);
      Em::Emit(Ec, h[0], tl, g0 + 2 * tid);
      uint32_t xr[1][4] = {{r[0], r[1], r[2], r[3]}};
      HashWords<1, BN, true>(xr, h, L);
      Em::Emit(Ec, h[0], tr, g0 + 2 * tid + 1);
    }
  }
  DPF_COOP_MARK(4);
}

template <int E, class Em>
int LaunchExpandCoop(hipStream_t st, const ExpandArgs& a, const VtDev& vt) {
  const int64_t cpk = a.chunk_end - a.chunk_begin;
  int64_t blocks = cpk;
  if (a.batched) {
    if constexpr (!Em::kCanBatch) {
      return SetError(DPF_AMD_INTERNAL, "batched expansion needs a directly convertible type");
    } else {
      blocks = cpk * a.num_keys;
      if (blocks < 1 || blocks > INT32_MAX)
        return SetError(DPF_AMD_INVALID_ARGUMENT, "batched expansion grid out of range");
      hipLaunchKernelGGL((KExpandCoop<E, Em, true>), dim3((unsigned)blocks), dim3(kCoopBlock), 0,
                         st, a, vt);
      return LaunchCheck("expand kernel launch");
    }
  }
  if (blocks < 1 || blocks > INT32_MAX)
    return SetError(DPF_AMD_INVALID_ARGUMENT, "expansion grid out of range");
  hipLaunchKernelGGL((KExpandCoop<E, Em, false>), dim3((unsigned)blocks), dim3(kCoopBlock), 0, st,
                     a, vt);
  return LaunchCheck("expand kernel launch");
}

// D in {0, 1, 2, 4, 5, 6, 8}: KExpand with DFS depth D; D = -1 / -2 / -3:
// KExpandCoop with E = 0 / 1 / -2.
template <class Em>
int LaunchExpandAnyD(int D, int grid, hipStream_t st, const ExpandArgs& a, const VtDev& vt) {
  if (D == -1) return LaunchExpandCoop<0, Em>(st, a, vt);
  if (D == -2) return LaunchExpandCoop<1, Em>(st, a, vt);
  if (D == -3) return LaunchExpandCoop<-2, Em>(st, a, vt);
  switch (D) {
    case 0:
      return LaunchExpand<0, Em>(grid, st, a, vt);
    case 1:
      return LaunchExpand<1, Em>(grid, st, a, vt);
    case 2:
      return LaunchExpand<2, Em>(grid, st, a, vt);
    case 4:
      return LaunchExpand<4, Em>(grid, st, a, vt);
    case 5:
      return LaunchExpand<5, Em>(grid, st, a, vt);
    case 6:
      return LaunchExpand<6, Em>(grid, st, a, vt);
#if DPF_EXPAND_EXTRA_DEPTHS  // A/B builds only (tools/ab_c3_depth.sh)
    case 3:
      return LaunchExpand<3, Em>(grid, st, a, vt);
#endif
    default:
      return LaunchExpand<8, Em>(grid, st, a, vt);
  }
}

}  // namespace dpf_amd
