// k_walk.hip — path-walk kernels: EvaluateSeeds (evaluate_prg_hwy.cc:552-634),
// the fused EvaluateAt / EvaluateAndApply point evaluation and the plain
// AES-MMO hash (aes_128_fixed_key_hash.cc:57-98).
//
// Both walks give each thread two points (i, i + T) walked in lockstep — two
// independent AES chains per lane keep the LDS fed — when the launch has
// more points than threads; a wave with no second point takes the one-state
// path (the choice is wave-uniform).  The left/right PRG key is chosen per
// lane from the path bit by masking the key difference into the state
// (DpfMasked / PairMasked), one AES per level as the Highway walk
// (evaluate_prg_hwy.cc:235-377).
#include "aes_device.h"

namespace dpf_amd {

__device__ __forceinline__ uint32_t PathBit(const uint4& p, int bit_index) {
  if (bit_index >= 128) return 0;
  uint32_t w = bit_index < 32 ? p.x : bit_index < 64 ? p.y : bit_index < 96 ? p.z : p.w;
  return (w >> (bit_index & 31)) & 1u;
}

// Per-lane choice between two generic keys of a kernel argument (the
// differences are SALU work on SGPR words).
template <int N>
struct PairMasked {
  const KeyPair& kp;
  uint32_t m[N];
  __device__ __forceinline__ uint32_t rk(int, int i) const { return kp.k[0].rk[i]; }
  __device__ __forceinline__ uint32_t rkr(int, int i) const { return kp.k[0].rkr[i]; }
  __device__ __forceinline__ uint32_t post(int n, int i, uint32_t w) const {
    return w ^ ((kp.k[0].rk[i] ^ kp.k[1].rk[i]) & m[n]);
  }
};

template <int N>
struct DpfMaskedKeys {
  __device__ __forceinline__ DpfMasked<N> operator()(const uint32_t (&m)[N]) const {
    DpfMasked<N> k;
#pragma unroll
    for (int n = 0; n < N; ++n) k.m[n] = m[n];
    return k;
  }
};
template <int N>
struct PairMaskedKeys {
  const KeyPair& kp;
  __device__ __forceinline__ PairMasked<N> operator()(const uint32_t (&m)[N]) const {
    PairMasked<N> k{kp, {}};
#pragma unroll
    for (int n = 0; n < N; ++n) k.m[n] = m[n];
    return k;
  }
};

// Progress-ordered wave priority for the lane-per-point walks: the
// sequencer serves a SIMD's older waves first, so the waves of a round of
// blocks finish one after another and the last ones run below the occupancy
// the LDS needs.  A wave starts at priority 3 and steps down one level per
// quarter of its levels, so the waves behind are served first (the scheme of
// KExpand's DPF_EXPAND_PRIO).  c2's batched 64-key launch 1.587-1.600 ->
// 1.555-1.577 ms (profiles/ab_walk_prio_r06x/); DPF_WALK_PRIO=0 turns it off.
#ifndef DPF_WALK_PRIO
#define DPF_WALK_PRIO 1
#endif
#ifndef DPF_DCF_PRIO
#define DPF_DCF_PRIO 1  // the same per hierarchy level in KDcfEvaluateDirect
#endif
__device__ __forceinline__ void WalkPrio(int level, int num_levels) {
  if constexpr (DPF_WALK_PRIO != 0) {
    if (num_levels < 8) return;
    const int q = (level * 4) / num_levels;  // wave-uniform
    if (level > 0 && q != ((level - 1) * 4) / num_levels) {
      if (q == 1)
        __builtin_amdgcn_s_setprio(2);
      else if (q == 2)
        __builtin_amdgcn_s_setprio(1);
      else
        __builtin_amdgcn_s_setprio(0);
    } else if (level == 0) {
      __builtin_amdgcn_s_setprio(3);
    }
  }
}

// NP points of one thread: their indices, the index of their per-seed (or
// per-key) inputs, and the walk state.
template <int NP>
struct Walk {
  int64_t idx[NP];
  int64_t src[NP];
  uint32_t x[NP][4];
  uint32_t t[NP];
};

// Walks NP points num_levels levels (EvaluateSeeds semantics: level l uses
// path bit num_levels - 1 - l + rightshift; correction words shared, per
// seed [level][seed], or per key [key][level]).
template <int NP, class KeyMaker>
__device__ __forceinline__ void WalkPoints(const WalkArgs& w, Walk<NP>& s, const KeyMaker& km,
                                           const Lds& L) {
  const int64_t ppk = w.points_per_key;
  const bool by_key = ppk > 0 || w.key_index != nullptr;
  const bool per_seed = !by_key && w.num_cw > w.num_levels;
  const int64_t cw_step = per_seed ? w.num_seeds : 1;
  int64_t cw_base[NP];
  uint4 p[NP];
#pragma unroll
  for (int n = 0; n < NP; ++n) {
    s.src[n] = w.key_index ? (int64_t)w.key_index[s.idx[n]] : ppk > 0 ? s.idx[n] / ppk : s.idx[n];
    cw_base[n] = by_key ? s.src[n] * w.num_levels : per_seed ? s.idx[n] : 0;
    const int64_t si = (ppk > 0 || (w.key_index && w.seeds_by_key)) ? s.src[n] : s.idx[n];
    const uint4 v = w.seeds_in[si];
    s.x[n][0] = v.x;
    s.x[n][1] = v.y;
    s.x[n][2] = v.z;
    s.x[n][3] = v.w;
    s.t[n] = w.cb_in[si];
    if (w.paths) {
      p[n] = w.paths[s.idx[n]];
    } else {  // implicit paths: point j of each key is tree index j
      const uint64_t j = (uint64_t)(ppk > 0 ? s.idx[n] - s.src[n] * ppk : s.idx[n]) +
                         (uint64_t)w.path_offset;
      p[n] = make_uint4((uint32_t)j, (uint32_t)(j >> 32), 0u, 0u);
    }
  }
  for (int level = 0; level < w.num_levels; ++level) {
    WalkPrio(level, w.num_levels);
    const int bi = w.num_levels - level - 1 + w.rightshift;
    uint32_t bit[NP], mask[NP];
    Cw cw[NP];
    uint32_t sg[NP][4], st[NP][4];
#pragma unroll
    for (int n = 0; n < NP; ++n) {
      bit[n] = PathBit(p[n], bi);
      mask[n] = 0u - bit[n];
      cw[n] = LoadCw(w.cw_seed, w.ccl, w.ccr, cw_base[n] + level * cw_step);
      Sigma(s.x[n], sg[n]);
#pragma unroll
      for (int c = 0; c < 4; ++c) st[n][c] = sg[n][c];
    }
    AesN<NP>(st, km(mask), L);
#pragma unroll
    for (int n = 0; n < NP; ++n) {
      const uint32_t m = 0u - s.t[n];
#pragma unroll
      for (int c = 0; c < 4; ++c) s.x[n][c] = st[n][c] ^ sg[n][c] ^ (cw[n].seed[c] & m);
      const uint32_t nt = (s.x[n][0] & 1u) ^ (s.t[n] & (bit[n] ? cw[n].cr : cw[n].cl));
      s.x[n][0] &= ~1u;
      s.t[n] = nt;
    }
  }
}

template <int NP>
__device__ __forceinline__ void StoreWalk(const WalkArgs& w, const Walk<NP>& s, int live) {
#pragma unroll
  for (int n = 0; n < NP; ++n) {
    if (n >= live) break;
    w.seeds_out[s.idx[n]] = make_uint4(s.x[n][0], s.x[n][1], s.x[n][2], s.x[n][3]);
    w.cb_out[s.idx[n]] = (uint8_t)s.t[n];
  }
}

// Generic-key EvaluateSeeds (evaluate_prg_hwy.cc:552-634).
template <int NP>
__device__ __forceinline__ void SeedsIter(const WalkArgs& w, const KeyPair& kp, const Lds& L,
                                          int64_t base, int64_t T) {
  Walk<NP> s;
  const int live = (NP == 2 && base + T < w.num_seeds) ? 2 : 1;
#pragma unroll
  for (int n = 0; n < NP; ++n) s.idx[n] = n < live ? base + n * T : base;
  WalkPoints<NP>(w, s, PairMaskedKeys<NP>{kp}, L);
  StoreWalk<NP>(w, s, live);
}

__global__ __launch_bounds__(kPointsBlock, kPointsWaves) void KEvaluateSeeds(WalkArgs a,
                                                                              KeyPair kp) {
  __shared__ uint32_t tab[kTabWords];
  FillTables(tab);
  __syncthreads();
  const Lds L = MakeLds(tab);
  const int64_t T = (int64_t)gridDim.x * blockDim.x;
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; base < a.num_seeds;
       base += 2 * T) {
    if (__ballot(base + T < a.num_seeds) != 0) {
      SeedsIter<2>(a, kp, L, base, T);
    } else {
      SeedsIter<1>(a, kp, L, base, T);
    }
  }
}

// EvaluateAtImpl / EvaluateAndApply per-point evaluation (h:1013-1063,
// 1143-1189): walk, value hash (HashExpandedSeeds), conversion + correction
// of element block_index[i].
template <int NP, int BN>
__device__ __forceinline__ void PointsIter(const PointsArgs& a, const VtDev& vt, const Lds& L,
                                           int64_t base, int64_t T) {
  const WalkArgs& w = a.w;
  Walk<NP> s;
  const int live = (NP == 2 && base + T < w.num_seeds) ? 2 : 1;
#pragma unroll
  for (int n = 0; n < NP; ++n) s.idx[n] = n < live ? base + n * T : base;
  WalkPoints<NP>(w, s, DpfMaskedKeys<NP>{}, L);
  if (w.seeds_out) StoreWalk<NP>(w, s, live);
  u128 W[NP][BN];
  if constexpr (NP * BN <= 4) {
    HashSeeds<NP, BN>(s.x, W, L);
  } else {
#pragma unroll
    for (int n = 0; n < NP; ++n) {
      const uint32_t xn[1][4] = {{s.x[n][0], s.x[n][1], s.x[n][2], s.x[n][3]}};
      u128 Wn[1][BN];
      HashSeeds<1, BN>(xn, Wn, L);
#pragma unroll
      for (int j = 0; j < BN; ++j) W[n][j] = Wn[0][j];
    }
  }
  const int per_elem = vt.epb * vt.ns;
#pragma unroll
  for (int n = 0; n < NP; ++n) {
    if (n >= live) break;
    const int bi = a.block_index ? a.block_index[s.idx[n]] : 0;
    const int party = a.party ? a.party[s.src[n]] : vt.party;
    char* dst = a.out + s.idx[n] * (int64_t)vt.stride;
    if (a.value_corrections) {
      u128 corr[kMaxCorrections];
      const uint4* c4 = a.value_corrections + s.src[n] * per_elem;
      for (int j = 0; j < per_elem; ++j) {
        const uint4 c = c4[j];
        corr[j] = (u128)c.x | ((u128)c.y << 32) | ((u128)c.z << 64) | ((u128)c.w << 96);
      }
      EmitLeaf<BN>(vt, W[n], s.t[n] != 0, party, corr, bi, bi + 1,
                   [dst](int) { return dst; });
    } else {
      EmitLeaf<BN>(vt, W[n], s.t[n] != 0, party, vt.corr, bi, bi + 1,
                   [dst](int) { return dst; });
    }
  }
}

// KEvaluatePoints<BN> for BN <= 2 runs one point chain per lane at 8
// waves/SIMD (1024-thread blocks, 52-57 VGPRs): c2 1.67 -> 1.57 ms against
// two chains per lane at 4 waves/SIMD (a kernel holding both paths needs
// 104 VGPRs); one chain at 6 waves was slower (1.74).  BN = 4 (94 VGPRs for
// one chain) keeps two chains per lane at 4 waves.
template <int BN>
constexpr bool kPointsTwoChains = BN > 2;
template <int BN>
constexpr int kPointsBlockOf = kPointsTwoChains<BN> ? kPointsBlock : 1024;
template <int BN>
constexpr int kPointsWavesOf = kPointsTwoChains<BN> ? kPointsWaves : 8;

template <int BN>
__global__ __launch_bounds__(kPointsBlockOf<BN>, kPointsWavesOf<BN>) void KEvaluatePoints(
    PointsArgs a, VtDev vt) {
  __shared__ uint32_t tab[kTabWords];
  FillTables(tab);
  __syncthreads();
  const Lds L = MakeLds(tab);
  const int64_t T = (int64_t)gridDim.x * blockDim.x;
  if constexpr (kPointsTwoChains<BN>) {
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; base < a.w.num_seeds;
         base += 2 * T) {
      if (__ballot(base + T < a.w.num_seeds) != 0) {
        PointsIter<2, BN>(a, vt, L, base, T);
      } else {
        PointsIter<1, BN>(a, vt, L, base, T);
      }
    }
  } else {
    for (int64_t base = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; base < a.w.num_seeds;
         base += T)
      PointsIter<1, BN>(a, vt, L, base, T);
  }
}

// ----------------------------------------------------------------------------
// Quad-lane walk for launches too small to fill the chip
// ----------------------------------------------------------------------------
//
// A point's walk is a chain of one AES per level (129 at log_domain 128), so
// a launch of a few thousand points (one key's EvaluateAt: 16,384 points =
// 256 waves, one per CU) runs at the latency of a lone wave's AES: the
// 16 v_perm + 16 ds_read_b32 + 12 combine ops of a round issue back to back
// from one wave (~350 cycles/round measured: 217 us per 129-level launch).
// Here four lanes share a point, lane c holding column c of the state:
// per round a lane forms its column from its own byte 0 and bytes 1-3 of the
// next three columns (three quad_perm DPP moves), i.e. 4 lookups + 3 moves +
// 5 VALU instead of 16 + 28, and the launch has four times the waves.  Round
// keys are per column, so each lane keeps its column's words of the left key,
// the left/right difference and the value key in registers (33 VGPRs).
// Semantics are those of PointsIter (walk, value hash, emit) for BN <= 2.

// T4: four 64 KiB-halved tables (aes_device.h FillTables4, 128 KiB per
// block), for launches of at most kQuadT4MaxPoints points (one block per CU).
#ifndef DPF_QUAD_AHEAD
#define DPF_QUAD_AHEAD 1
#endif
// Phase timestamps of KEvaluatePointsQuad (diagnostic builds only,
// DPF_QUAD_TRACE=1, tools/quad_trace.py): per block, thread 0's s_memtime
// (shader clock) and s_memrealtime (100 MHz) at entry, after the tables,
// after the walk and at the end.
#if DPF_QUAD_TRACE
__device__ uint64_t g_quad_trace[4096 * 8];
#define DPF_QUAD_MARK(i)                                                     \
  do {                                                                       \
    if (threadIdx.x == 0 && blockIdx.x < 4096) {                             \
      g_quad_trace[blockIdx.x * 8 + 2 * (i)] = __builtin_amdgcn_s_memtime();  \
      g_quad_trace[blockIdx.x * 8 + 2 * (i) + 1] = __builtin_amdgcn_s_memrealtime(); \
    }                                                                        \
  } while (0)
extern "C" __attribute__((visibility("default"))) int dpf_amd_debug_quad_trace(void* host,
                                                                               int64_t bytes) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_quad_trace), (size_t)bytes, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : 1;
}
#else
#define DPF_QUAD_MARK(i) \
  do {                   \
  } while (0)
#endif
template <int BN, bool T4>
__global__ __launch_bounds__(kPointsBlock, kPointsWaves) void KEvaluatePointsQuad(PointsArgs a,
                                                                                   VtDev vt) {
  __shared__ uint32_t tab[T4 ? kTab4Words : kTabWords];
  DPF_QUAD_MARK(0);
  // The lane's first point is read before the table fill: `paths` may be a
  // pinned host slot mapped into the device (one EvaluateAt call's points,
  // read in place), whose PCIe round trip then overlaps the fill.
  const int64_t i_first = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2;
  uint4 p_first = make_uint4(0u, 0u, 0u, 0u);
  uint32_t x_first = 0u, t_first = 0u;  // its seed word and control bit (no key index)
  if (i_first < a.w.num_seeds) {
    if (a.w.paths) p_first = a.w.paths[i_first];
    if (a.w.key_index == nullptr) {
      const int64_t si0 = a.w.points_per_key > 0 ? i_first / a.w.points_per_key : i_first;
      x_first = reinterpret_cast<const uint32_t*>(a.w.seeds_in)[si0 * 4 + (threadIdx.x & 3)];
      t_first = a.w.cb_in[si0];
    }
  }
  if constexpr (T4)
    FillTables4(tab);
  else
    FillTables(tab);
  __syncthreads();
  DPF_QUAD_MARK(1);
  using LT = std::conditional_t<T4, Lds4, Lds>;
  LT L;
  if constexpr (T4)
    L = MakeLds4(tab);
  else
    L = MakeLds(tab);
  const int c = threadIdx.x & 3;
  const QuadKey kl = MakeQuadKey<0>(c), kv = MakeQuadKey<2>(c);
  const QuadRk klr = MakeQuadRk<0>(c), kvr = MakeQuadRk<2>(c);
  const QuadDiff kd = MakeQuadDiff(c);
  const WalkArgs& w = a.w;
  const int64_t ppk = w.points_per_key;
  const bool by_key = ppk > 0 || w.key_index != nullptr;
  const bool per_seed = !by_key && w.num_cw > w.num_levels;
  const int64_t cw_step = per_seed ? w.num_seeds : 1;
  const uint32_t* cw_words = reinterpret_cast<const uint32_t*>(w.cw_seed);
  const int per_elem = vt.epb * vt.ns;
  const int64_t T = ((int64_t)gridDim.x * blockDim.x) >> 2;
  for (int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 2; i < w.num_seeds;
       i += T) {
    const int64_t src = w.key_index ? (int64_t)w.key_index[i] : ppk > 0 ? i / ppk : i;
    const int64_t cw_base = by_key ? src * w.num_levels : per_seed ? i : 0;
    const int64_t si = (ppk > 0 || (w.key_index && w.seeds_by_key)) ? src : i;
    const bool first = i == i_first && w.key_index == nullptr;
    uint32_t x = first ? x_first : reinterpret_cast<const uint32_t*>(w.seeds_in)[si * 4 + c];
    uint32_t t = first ? t_first : w.cb_in[si];
    uint4 p;
    if (w.paths) {
      p = i == i_first ? p_first : w.paths[i];
    } else {
      const uint64_t j = (uint64_t)(ppk > 0 ? i - src * ppk : i) + (uint64_t)w.path_offset;
      p = make_uint4((uint32_t)j, (uint32_t)(j >> 32), 0u, 0u);
    }
#if DPF_QUAD_AHEAD
    // A level is ~1,100 cycles of dependent rounds: its correction word and
    // path bit are loaded / formed one level ahead, off the chain, and the
    // path sits in a shift register whose top bit is the next level's bit
    // (PathBit's uniform word choice compiled to a branch tree in the loop).
    const int nl = w.num_levels;
    const int top = nl + w.rightshift;  // path bits [rightshift, top) are walked, msb first
    u128 pp = (u128)p.x | ((u128)p.y << 32) | ((u128)p.z << 64) | ((u128)p.w << 96);
    if (top > 128)
      pp >>= (top - 128);  // the levels above bit 127 walk zeros (PathBit)
    else if (top > 0 && top < 128)
      pp <<= (128 - top);
    int64_t ci = cw_base;
    uint32_t cw_n = nl > 0 ? cw_words[ci * 4 + c] : 0u;
    uint32_t cl_n = nl > 0 ? w.ccl[ci] : 0u, cr_n = nl > 0 ? w.ccr[ci] : 0u;
    for (int level = 0; level < nl; ++level) {
      const uint32_t cwc = cw_n, cl = cl_n, cr = cr_n;
      const uint32_t bit = (uint32_t)(pp >> 127);
      pp <<= 1;
      if (level + 1 < nl) ci += cw_step;
      cw_n = cw_words[ci * 4 + c];
      cl_n = w.ccl[ci];
      cr_n = w.ccr[ci];
      if constexpr (T4 || DPF_QUAD_RKM)
        QuadWalkStepRk<T4>(x, t, bit, cwc, cl, cr, c, klr, kd, L);
      else
        QuadWalkStep(x, t, bit, cwc, cl, cr, c, kl, kd, L);
    }
#else
    for (int level = 0; level < w.num_levels; ++level) {
      const uint32_t bit = PathBit(p, w.num_levels - level - 1 + w.rightshift);
      const int64_t ci = cw_base + level * cw_step;
      if constexpr (T4 || DPF_QUAD_RKM)
        QuadWalkStepRk<T4>(x, t, bit, cw_words[ci * 4 + c], w.ccl[ci], w.ccr[ci], c, klr, kd, L);
      else
        QuadWalkStep(x, t, bit, cw_words[ci * 4 + c], w.ccl[ci], w.ccr[ci], c, kl, kd, L);
    }
#endif
    DPF_QUAD_MARK(2);
    if (w.seeds_out) {
      reinterpret_cast<uint32_t*>(w.seeds_out)[i * 4 + c] = x;
      if (c == 0) w.cb_out[i] = (uint8_t)t;
    }
    if (a.out == nullptr) continue;  // a walk only (EvaluateSeeds): no value hash
    // value hash (HashExpandedSeeds, cc:523-547): blocks H_V(seed + j), a
    // 128-bit add (a walk of zero levels leaves the key's seed, bit 0 set or
    // not)
    u128 W[BN];
#pragma unroll
    for (int j = 0; j < BN; ++j) {
      uint32_t in = x;
      if (j > 0) {
        const u128 v = ((u128)QuadPerm<kQuadBcast<0>>(x) | ((u128)QuadPerm<kQuadBcast<1>>(x) << 32) |
                        ((u128)QuadPerm<kQuadBcast<2>>(x) << 64) |
                        ((u128)QuadPerm<kQuadBcast<3>>(x) << 96)) +
                       (u128)j;
        in = (uint32_t)(v >> (32 * c));
      }
      const uint32_t sg = SigmaQuad(in, c);
      uint32_t h;
      if constexpr (T4 || DPF_QUAD_RKM)
        h = AesQuadRk<T4>(sg, kvr, L) ^ sg;
      else
        h = AesQuad<false>(sg, kv, kd, 0u, L) ^ sg;
      const uint32_t h0 = QuadPerm<kQuadBcast<0>>(h), h1 = QuadPerm<kQuadBcast<1>>(h),
                     h2 = QuadPerm<kQuadBcast<2>>(h), h3 = QuadPerm<kQuadBcast<3>>(h);
      W[j] = (u128)h0 | ((u128)h1 << 32) | ((u128)h2 << 64) | ((u128)h3 << 96);
    }
    if (c != 0) continue;
    const int bi = a.block_index ? a.block_index[i] : 0;
    const int party = a.party ? a.party[src] : vt.party;
    char* dst = a.out + i * (int64_t)vt.stride;
    if (a.value_corrections) {
      u128 corr[kMaxCorrections];
      const uint4* c4 = a.value_corrections + src * per_elem;
      for (int j = 0; j < per_elem; ++j) {
        const uint4 cc = c4[j];
        corr[j] = (u128)cc.x | ((u128)cc.y << 32) | ((u128)cc.z << 64) | ((u128)cc.w << 96);
      }
      EmitLeaf<BN>(vt, W, t != 0, party, corr, bi, bi + 1, [dst](int) { return dst; });
    } else {
      EmitLeaf<BN>(vt, W, t != 0, party, vt.corr, bi, bi + 1, [dst](int) { return dst; });
    }
    DPF_QUAD_MARK(3);
  }
}

// Up to 8192 blocks: past one resident round the dispatcher back-fills CUs
// that finish early (c2 batched: 1.69 ms at 8192 vs 1.82 ms capped at 512).
// Threads walk a second point only beyond 8192 blocks' worth of points.
#ifndef DPF_WALK_MAX_GRID
#define DPF_WALK_MAX_GRID 8192
#endif

// Threads per block for a walk over n points: full blocks once the launch
// fills every CU (two blocks each), smaller ones before that so that small
// launches still spread over all CUs.
static int WalkBlock(int64_t n, int max_block = kPointsBlock) {
  int64_t per = (n + 2 * 256 - 1) / (2 * 256);
  per = (per + 63) / 64 * 64;
  return (int)std::min<int64_t>(max_block, std::max<int64_t>(64, per));
}

// Little-endian load of an `nbytes` scalar.
__device__ __forceinline__ u128 LoadScalar(const char* p, int nbytes) {
  u128 v = 0;
  for (int b = nbytes - 1; b >= 0; --b) v = (v << 8) | (uint8_t)p[b];
  return v;
}

// Fused DCF BatchEvaluate: one walk per (key i, point i) through all tree
// levels; at hierarchy level h (log domain h, tree level tree_of[h]) the
// level's output is needed only when DCF bit (log_domain - h - 1) of the
// point is 0 (h:150-165 adds it then), so only those levels are hashed,
// converted, corrected and summed with the value type's + (the skipped
// levels' outputs are never read, so the result is identical).  Path bit of
// tree level a: log_domain - 1 - a (EvaluateAndApply rightshift 1).
// One value block (61 VGPRs): DPF_DCF_WAVES1 waves/SIMD.
#ifndef DPF_DCF_MAX_GRID
#define DPF_DCF_MAX_GRID 1024
#endif
#ifndef DPF_DCF_WAVES1
#define DPF_DCF_WAVES1 8  // c5-style DCF (uint64): 1.38 -> 1.25 ms at 2^20 evaluations
#endif
template <int BN>
constexpr int kDcfBlockOf = BN == 1 ? 128 * DPF_DCF_WAVES1 : kPointsBlock;
template <int BN>
constexpr int kDcfWavesOf = BN == 1 ? DPF_DCF_WAVES1 : kPointsWaves;

template <int BN>
__global__ __launch_bounds__(kDcfBlockOf<BN>, kDcfWavesOf<BN>) void KDcfEvaluate(DcfArgs a,
                                                                                 VtDev vt) {
  __shared__ uint32_t tab[kTabWords];
  FillTables(tab);
  __syncthreads();
  const Lds L = MakeLds(tab);
  const int64_t T = (int64_t)gridDim.x * blockDim.x;
  const int per_elem = vt.epb * vt.ns;
  const int H = a.log_domain;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += T) {
    const uint4 s0 = a.seeds[i];
    uint32_t x[1][4] = {{s0.x, s0.y, s0.z, s0.w}};
    uint32_t t = a.cb[i];
    const uint4 p = a.points[i];
    const u128 pv = (u128)p.x | ((u128)p.y << 32) | ((u128)p.z << 64) | ((u128)p.w << 96);
    const int party = a.party[i];
    u128 acc[DPF_AMD_MAX_SCALARS];
    for (int s = 0; s < vt.ns; ++s) acc[s] = 0;
    int level = 0;
    for (int h = 0; h < H; ++h) {
      if (DPF_DCF_PRIO) WalkPrio(h, H);
      const int stop = a.tree_of[h];
      for (; level < stop; ++level) {
        const uint32_t bit = PathBit(p, H - 1 - level);
        const Cw cw = LoadCw(a.cw_seed, a.ccl, a.ccr, (int64_t)level * a.n + i);
        WalkStep(x[0], t, bit, cw, DpfMasked<1>{{0u - bit}}, L);
      }
      if (PathBit(p, H - 1 - h) != 0) continue;
      u128 W[1][BN];
      HashSeeds<1, BN>(x, W, L);
      const int bbits = h - stop;
      const int e = bbits > 0 ? (int)((pv >> (H - h)) & (((u128)1 << bbits) - 1)) : 0;
      u128 corr[kMaxCorrections];
      const uint4* c4 = a.corrections + ((int64_t)h * a.n + i) * per_elem;
      for (int j = 0; j < per_elem; ++j) {
        const uint4 c = c4[j];
        corr[j] = (u128)c.x | ((u128)c.y << 32) | ((u128)c.z << 64) | ((u128)c.w << 96);
      }
      alignas(16) char buf[DPF_AMD_MAX_SCALARS * 16];
      char* dst = buf;
      EmitLeaf<BN>(vt, W[0], t != 0, party, corr, e, e + 1, [dst](int) { return dst; });
      for (int s = 0; s < vt.ns; ++s)
        acc[s] = ScAdd(vt.sc[s], acc[s], LoadScalar(buf + vt.sc[s].out_off, vt.sc[s].bytes));
    }
    char* out = a.out + i * (int64_t)vt.stride;
    for (int s = 0; s < vt.ns; ++s) StoreScalar(out + vt.sc[s].out_off, vt.sc[s].bytes, acc[s]);
  }
}

// KDcfEvaluate for a single integer / XorWrapper scalar of B bytes (uint64
// DCFs, the reference's BM_EvaluateDcf shape): the element, its correction,
// the negation and the sum stay in registers (U = uint64 up to 8 bytes,
// u128 for 16) — the generic kernel stages each level's element through a
// byte buffer and indexes its correction and accumulator arrays at run
// time, which lands them in scratch (1 KiB per lane).
#ifndef DPF_DCF_QUEUE
#define DPF_DCF_QUEUE 3  // queued value hashes per lane (0: in place; 2^20 uint64: 0.88 / 0.86 / 0.82 ms at 0 / 2 / 3)
#endif
template <bool XOR, int B>
__global__ __launch_bounds__(kDcfBlockOf<1>, kDcfWavesOf<1>) void KDcfEvaluateDirect(DcfArgs a,
                                                                                    VtDev vt) {
  using U = typename std::conditional<(B > 8), u128, uint64_t>::type;
  __shared__ uint32_t tab[kTabWords];
  FillTables(tab);
  __syncthreads();
  const Lds L = MakeLds(tab);
  const int64_t T = (int64_t)gridDim.x * blockDim.x;
  const int per_elem = vt.epb;
  const int H = a.log_domain;
  const U mask = B >= (int)sizeof(U) ? ~(U)0 : (((U)1 << (8 * B)) - 1);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += T) {
    const uint4 s0 = a.seeds[i];
    uint32_t x[4] = {s0.x, s0.y, s0.z, s0.w};
    uint32_t t = a.cb[i];
    const uint4 p = a.points[i];
    const u128 pv = (u128)p.x | ((u128)p.y << 32) | ((u128)p.z << 64) | ((u128)p.w << 96);
    const bool negate = a.party[i] == 1;
    U acc = 0;
    // hashes the seed of hierarchy level h (control bit tt) and adds the
    // corrected element to acc
    // element index of hierarchy level h within its block (h is wave-uniform)
    auto elem_of = [&](int h) {
      const int bbits = h - a.tree_of[h];
      return bbits > 0 ? (int)((pv >> (H - h)) & (((u128)1 << bbits) - 1)) : 0;
    };
    auto add_level = [&](const uint32_t (&xs)[1][4], uint32_t tt, int h, int e) {
      u128 W[1][1];
      HashSeeds<1, 1>(xs, W, L);
      U v = (U)(W[0][0] >> (8 * B * e)) & mask;
      const uint4 c = a.corrections[((int64_t)h * a.n + i) * per_elem + e];
      const U corr =
          (U)((u128)c.x | ((u128)c.y << 32) | ((u128)c.z << 64) | ((u128)c.w << 96)) & mask;
      if (XOR) {
        if (tt) v ^= corr;
        acc ^= v;  // XorWrapper: -v = v
      } else {
        if (tt) v = (v + corr) & mask;
        acc = (negate ? acc - v : acc + v) & mask;
      }
    };
#if DPF_DCF_QUEUE > 0
    // A lane needs the hash of about half the levels, and a wave ran every
    // level any of its lanes needed (~32 of the 47 algorithmic AES idle).
    // Here a lane queues the seeds it needs (up to DPF_DCF_QUEUE in
    // registers) and the wave hashes one queued seed per lane only when every
    // lane has one or some lane's queue is full; the rest drain at the end.
    // Integer + and XOR are commutative, so the order of the additions does
    // not change the result.
    constexpr int KQ = DPF_DCF_QUEUE;
    uint32_t qx[KQ][4], qm[KQ];
    int cnt = 0;
    auto pop = [&]() {
      if (cnt > 0) {
        const uint32_t xs[1][4] = {{qx[0][0], qx[0][1], qx[0][2], qx[0][3]}};
        add_level(xs, qm[0] >> 16, (int)(qm[0] & 255u), (int)((qm[0] >> 8) & 255u));
#pragma unroll
        for (int k = 0; k + 1 < KQ; ++k) {
#pragma unroll
          for (int c = 0; c < 4; ++c) qx[k][c] = qx[k + 1][c];
          qm[k] = qm[k + 1];
        }
        --cnt;
      }
    };
#endif
    int level = 0;
    for (int h = 0; h < H; ++h) {
      const int stop = a.tree_of[h];
      for (; level < stop; ++level) {
        const uint32_t bit = PathBit(p, H - 1 - level);
        const Cw cw = LoadCw(a.cw_seed, a.ccl, a.ccr, (int64_t)level * a.n + i);
        WalkStep(x, t, bit, cw, DpfMasked<1>{{0u - bit}}, L);
      }
#if DPF_DCF_QUEUE > 0
      if (PathBit(p, H - 1 - h) == 0) {
#pragma unroll
        for (int k = 0; k < KQ; ++k)
          if (cnt == k) {
#pragma unroll
            for (int c = 0; c < 4; ++c) qx[k][c] = x[c];
            qm[k] = (uint32_t)h | ((uint32_t)elem_of(h) << 8) | (t << 16);
          }
        ++cnt;
      }
      // wave-uniform: pop while every active lane holds a seed or a queue is full
      while (__builtin_amdgcn_ballot_w64(cnt == 0) == 0 ||
             __builtin_amdgcn_ballot_w64(cnt == KQ) != 0)
        pop();
#else
      if (PathBit(p, H - 1 - h) != 0) continue;
      const uint32_t xs[1][4] = {{x[0], x[1], x[2], x[3]}};
      add_level(xs, t, h, elem_of(h));
#endif
    }
#if DPF_DCF_QUEUE > 0
    while (__builtin_amdgcn_ballot_w64(cnt > 0) != 0) pop();
#endif
    char* out = a.out + i * (int64_t)vt.stride;
    StoreScalar(out + vt.sc[0].out_off, B, (u128)acc);
  }
}

template <bool XOR, int B>
static void LaunchDcfDirect(hipStream_t st, const DcfArgs& a, const VtDev& vt) {
  const int block = WalkBlock(a.n, kDcfBlockOf<1>);
  const int grid = (int)std::min<int64_t>(DPF_DCF_MAX_GRID, (a.n + block - 1) / block);
  hipLaunchKernelGGL((KDcfEvaluateDirect<XOR, B>), dim3(grid), dim3(block), 0, st, a, vt);
}

template <int BN>
static void LaunchDcf(hipStream_t st, const DcfArgs& a, const VtDev& vt) {
  const int block = WalkBlock(a.n, kDcfBlockOf<BN>);
  const int grid = (int)std::min<int64_t>(DPF_DCF_MAX_GRID, (a.n + block - 1) / block);
  hipLaunchKernelGGL((KDcfEvaluate<BN>), dim3(grid), dim3(block), 0, st, a, vt);
}

int LaunchDcfEvaluate(int bn, hipStream_t st, const DcfArgs& a, const VtDev& vt) {
  const ScalarDev& s0 = vt.sc[0];
  const bool one_direct = vt.direct && vt.ns == 1 && bn == 1 && s0.in_off == 0 &&
                          vt.esz == s0.bytes &&
                          (s0.kind == DPF_AMD_KIND_INTEGER || s0.kind == DPF_AMD_KIND_XOR_WRAPPER);
  if (one_direct && DcfDirectEnabled()) {
    const bool x = s0.kind == DPF_AMD_KIND_XOR_WRAPPER;
    switch (s0.bytes) {
      case 1:
        x ? LaunchDcfDirect<true, 1>(st, a, vt) : LaunchDcfDirect<false, 1>(st, a, vt);
        return LaunchCheck("dcf kernel launch");
      case 2:
        x ? LaunchDcfDirect<true, 2>(st, a, vt) : LaunchDcfDirect<false, 2>(st, a, vt);
        return LaunchCheck("dcf kernel launch");
      case 4:
        x ? LaunchDcfDirect<true, 4>(st, a, vt) : LaunchDcfDirect<false, 4>(st, a, vt);
        return LaunchCheck("dcf kernel launch");
      case 8:
        x ? LaunchDcfDirect<true, 8>(st, a, vt) : LaunchDcfDirect<false, 8>(st, a, vt);
        return LaunchCheck("dcf kernel launch");
      case 16:
        x ? LaunchDcfDirect<true, 16>(st, a, vt) : LaunchDcfDirect<false, 16>(st, a, vt);
        return LaunchCheck("dcf kernel launch");
      default:
        break;
    }
  }
  switch (bn) {
    case 1:
      LaunchDcf<1>(st, a, vt);
      break;
    case 2:
      LaunchDcf<2>(st, a, vt);
      break;
    default:
      LaunchDcf<4>(st, a, vt);
  }
  return LaunchCheck("dcf kernel launch");
}

// Plain AES-MMO hash (Aes128FixedKeyHash::Evaluate).
__global__ __launch_bounds__(kBlock, 2) void KAesMmo(const uint4* in, uint4* out, int64_t n,
                                                 KeyPair kp) {
  __shared__ uint32_t tab[kTabWords];
  FillTables(tab);
  __syncthreads();
  const Lds L = MakeLds(tab);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    uint4 v = in[i];
    uint32_t x[4] = {v.x, v.y, v.z, v.w}, s[4], st[1][4];
    Sigma(x, s);
#pragma unroll
    for (int c = 0; c < 4; ++c) st[0][c] = s[c];
    AesN<1>(st, PairSelect{{}, kp, false}, L);
    out[i] = make_uint4(st[0][0] ^ s[0], st[0][1] ^ s[1], st[0][2] ^ s[2], st[0][3] ^ s[3]);
  }
}

// EvaluateUntil's per-prefix roots (dpf.cc): prefix i
// starts from the partial evaluation of its tree index (row idx[i] of
// seeds / cb, written by the context walk) and walks `walk` (< 8, the
// previous level's log2(elements per block)) more levels along the low bits
// low[i] — the prefix's own node, which EvaluateUntil then expands.  Indices
// come from the host and are in range by construction; they are clamped so a
// corrupted one cannot read outside.
__global__ __launch_bounds__(256, 2) void KPrefixRoots(int64_t n, const int32_t* idx,
                                                       const uint8_t* low, int walk,
                                                       int64_t num_src, const uint4* seeds,
                                                       const uint8_t* cb, const uint4* cw_seed,
                                                       const uint8_t* ccl, const uint8_t* ccr,
                                                       uint4* seeds_out, uint8_t* cb_out) {
  __shared__ uint32_t tab[kTabWords];
  if (walk > 0) {  // kernel-uniform
    FillTables(tab);
    __syncthreads();
  }
  const Lds L = MakeLds(tab);
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step) {
    int64_t j = idx[i];
    j = j < 0 ? 0 : j >= num_src ? num_src - 1 : j;
    const uint4 s = seeds[j];
    uint32_t x[4] = {s.x, s.y, s.z, s.w};
    uint32_t t = cb[j];
    const uint32_t bits = low[i];
    for (int l = 0; l < walk; ++l) {
      const uint32_t bit = (bits >> (walk - 1 - l)) & 1u;
      WalkStep(x, t, bit, LoadCw(cw_seed, ccl, ccr, l), DpfMasked<1>{{0u - bit}}, L);
    }
    seeds_out[i] = make_uint4(x[0], x[1], x[2], x[3]);
    cb_out[i] = (uint8_t)t;
  }
}

int PrefixRoots(int64_t n, const int32_t* idx, const uint8_t* low, int walk, int64_t num_src,
                const void* seeds, const uint8_t* cb, const void* cw_seed, const uint8_t* ccl,
                const uint8_t* ccr, void* seeds_out, uint8_t* cb_out, void* stream) {
  if (n <= 0) return DPF_AMD_OK;
  if (num_src <= 0 || walk < 0 || walk > 7)
    return SetError(DPF_AMD_INTERNAL, "bad prefix roots arguments");
  const int grid = (int)std::min<int64_t>(1024, (n + 255) / 256);
  hipLaunchKernelGGL(KPrefixRoots, dim3(grid), dim3(256), 0, (hipStream_t)stream, n, idx, low,
                     walk, num_src, (const uint4*)seeds, cb, (const uint4*)cw_seed, ccl, ccr,
                     (uint4*)seeds_out, cb_out);
  return LaunchCheck("prefix roots kernel launch");
}

int LaunchEvaluateSeeds(int64_t n, hipStream_t st, const WalkArgs& a, const KeyPair& kp) {
  const int block = WalkBlock(n);
  const int grid = (int)std::min<int64_t>(DPF_WALK_MAX_GRID, (n + block - 1) / block);
  hipLaunchKernelGGL(KEvaluateSeeds, dim3(grid), dim3(block), 0, st, a, kp);
  return LaunchCheck("evaluate_seeds kernel launch");
}

template <int BN>
static void LaunchPoints(int64_t n, hipStream_t st, const PointsArgs& a, const VtDev& vt) {
  const int block = WalkBlock(n, kPointsBlockOf<BN>);
  const int grid = (int)std::min<int64_t>(DPF_WALK_MAX_GRID, (n + block - 1) / block);
  hipLaunchKernelGGL((KEvaluatePoints<BN>), dim3(grid), dim3(block), 0, st, a, vt);
}

// Four-table quad walk up to this many points: one 128 KiB-table block per
// CU holds the launch (<= 512 lanes per CU) in one resident round.
#ifndef DPF_QUAD_T4_MAX
#define DPF_QUAD_T4_MAX (256 * kPointsBlock / 4)
#endif
template <int BN>
static void LaunchPointsQuad(int64_t n, hipStream_t st, const PointsArgs& a, const VtDev& vt) {
  if (n <= DPF_QUAD_T4_MAX) {
    // one block per CU: 4n lanes over 256 blocks
    const int64_t per = ((4 * n + 255) / 256 + 63) / 64 * 64;
    const int block = (int)std::min<int64_t>(kPointsBlock, std::max<int64_t>(64, per));
    const int grid = (int)std::min<int64_t>(DPF_WALK_MAX_GRID, (4 * n + block - 1) / block);
    hipLaunchKernelGGL((KEvaluatePointsQuad<BN, true>), dim3(grid), dim3(block), 0, st, a, vt);
    return;
  }
  const int block = WalkBlock(4 * n, kPointsBlock);
  const int grid = (int)std::min<int64_t>(DPF_WALK_MAX_GRID, (4 * n + block - 1) / block);
  hipLaunchKernelGGL((KEvaluatePointsQuad<BN, false>), dim3(grid), dim3(block), 0, st, a, vt);
}

// Points below which the quad-lane walk runs (one-chain lanes fill the chip
// from ~2^18 points).
#ifndef DPF_WALK_QUAD_MAX
#define DPF_WALK_QUAD_MAX (1 << 16)
#endif

// EvaluateSeeds with the DPF's own PRG keys (the kernel's built-in key
// schedule).  A launch too small to fill the chip — the walk of a
// heavy-hitters level's 2^16 unique prefixes, 8 levels each — runs four lanes
// per seed (KEvaluatePointsQuad without the value hash) instead of a lone
// lane's 16-lookup rounds; larger ones keep the generic kernel.
int LaunchEvaluateSeedsDpf(int64_t n, hipStream_t st, const WalkArgs& a, const KeyPair& kp) {
  const int mode = WalkMode();  // 0 automatic, 1 quad-lane, 2 one lane per seed
  if (mode == 1 || (mode == 0 && n <= DPF_WALK_QUAD_MAX)) {
    PointsArgs pa{};
    pa.w = a;
    pa.out = nullptr;
    LaunchPointsQuad<1>(n, st, pa, VtDev{});
    return LaunchCheck("evaluate_seeds kernel launch");
  }
  return LaunchEvaluateSeeds(n, st, a, kp);
}

int LaunchEvaluatePoints(int bn, int64_t n, hipStream_t st, const PointsArgs& a,
                         const VtDev& vt) {
  const int mode = WalkMode();  // 0 automatic, 1 quad-lane, 2 one lane per point
  if (bn <= 2 && (mode == 1 || (mode == 0 && n <= DPF_WALK_QUAD_MAX))) {
    if (bn == 1)
      LaunchPointsQuad<1>(n, st, a, vt);
    else
      LaunchPointsQuad<2>(n, st, a, vt);
    return LaunchCheck("evaluate_points kernel launch");
  }
  switch (bn) {
    case 1:
      LaunchPoints<1>(n, st, a, vt);
      break;
    case 2:
      LaunchPoints<2>(n, st, a, vt);
      break;
    default:
      LaunchPoints<4>(n, st, a, vt);
  }
  return LaunchCheck("evaluate_points kernel launch");
}

int LaunchAesMmo(int grid, hipStream_t st, const uint4* in, uint4* out, int64_t n,
                 const KeyPair& kp) {
  hipLaunchKernelGGL(KAesMmo, dim3(grid), dim3(kBlock), 0, st, in, out, n, kp);
  return LaunchCheck("aes kernel launch");
}

}  // namespace dpf_amd
