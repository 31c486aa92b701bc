// dpf_kernels.hip — gfx950 kernels of the DPF tree expansion + dense-PIR scan
// hot path, and the Tier-1 C ABI that launches them (include/dpf_amd.h).
//
// AES design: CDNA4 has no AES instructions, so AES-128 runs
// as T-table lookups from LDS.  One 64 KiB table per workgroup holds, for each
// of the 256 byte values e, a 256-byte row [T0[e] x 32 | T1[e] x 32]: lane l
// reads replica (l & 31), i.e. bank (l & 31), so every ds_read_b32 is
// bank-conflict free whatever the data.  The row address is built with ONE
// v_perm_b32 (state byte -> address bits 8..15, lane offset -> bits 0..7);
// T1 is the same address + 128 (ds_read offset field), T2/T3 are rotations
// of T0/T1 folded into one v_alignbit per column.  Per round and column:
// 4 v_perm + 4 ds_read_b32 + 3 VALU; the round keys are SGPR constants.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>

#include "aes_tables.h"
#include "dpf_amd.h"
#include "internal.h"

namespace dpf_amd {

constexpr int kTabWords = 256 * 64;  // 64 KiB
constexpr int kBlock = 256;  // 64 KiB LDS table per block; 2 blocks per CU

__constant__ Te0Table c_te0 = MakeTe0();

struct KeyPair {
  AesKey k[2];
};

// ----------------------------------------------------------------------------
// AES core
// ----------------------------------------------------------------------------

struct Lds {
  const char* base;
  uint32_t laneoff;
};

__device__ __forceinline__ void FillTables(uint32_t* tab) {
  for (int i = threadIdx.x; i < kTabWords; i += blockDim.x) {
    uint32_t v = c_te0.t[i >> 6];
    tab[i] = (i & 32) ? ((v << 8) | (v >> 24)) : v;  // T1 = rotl8(T0)
  }
}

__device__ __forceinline__ Lds MakeLds(const uint32_t* tab) {
  return Lds{reinterpret_cast<const char*>(tab), (threadIdx.x & 31u) * 4u};
}

// Byte k of x to address bits 8..15, lane offset to bits 0..7.
#define DPF_SEL(k) (0x0c0c0000u | ((4u + (k)) << 8))

__device__ __forceinline__ uint32_t LoadT0(const Lds& L, uint32_t x, int k) {
  uint32_t a = __builtin_amdgcn_perm(x, L.laneoff, DPF_SEL(k));
  return *reinterpret_cast<const uint32_t*>(L.base + a);
}
__device__ __forceinline__ uint32_t LoadT1(const Lds& L, uint32_t x, int k) {
  uint32_t a = __builtin_amdgcn_perm(x, L.laneoff, DPF_SEL(k));
  return *reinterpret_cast<const uint32_t*>(L.base + a + 128);
}
__device__ __forceinline__ uint32_t Rotl16(uint32_t x) {
  return __builtin_amdgcn_alignbit(x, x, 16);
}

__device__ __forceinline__ uint32_t Xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // one v_bitop3_b32
}

// The three DPF PRG keys (cc:55-60) expanded at compile time.  Device code
// indexes them with unrolled constant indices, so every round-key word is a
// literal materialised by s_mov (SALU) next to its use: no constant-memory
// loads, no SGPR pressure, no VGPR-lane spills of hoisted keys.
constexpr AesKey kDpfKeys[3] = {ExpandAesKey(kPrgKeyLeftLo, kPrgKeyLeftHi),
                                ExpandAesKey(kPrgKeyRightLo, kPrgKeyRightHi),
                                ExpandAesKey(kPrgKeyValueLo, kPrgKeyValueHi)};

// Key accessors: rk(n, i) / rkr(n, i) for state n, round-key word i.
template <int W>
struct DpfKeyAt {  // one fixed DPF key for all states
  __device__ __forceinline__ uint32_t rk(int, int i) const { return kDpfKeys[W].rk[i]; }
  __device__ __forceinline__ uint32_t rkr(int, int i) const { return kDpfKeys[W].rkr[i]; }
};
struct DpfLeftRight {  // state 0: left key, state 1: right key
  __device__ __forceinline__ uint32_t rk(int n, int i) const { return kDpfKeys[n].rk[i]; }
  __device__ __forceinline__ uint32_t rkr(int n, int i) const { return kDpfKeys[n].rkr[i]; }
};
struct DpfSelect {  // per-lane choice of the left / right key (path walk)
  bool right;
  __device__ __forceinline__ uint32_t rk(int, int i) const {
    return right ? kDpfKeys[1].rk[i] : kDpfKeys[0].rk[i];
  }
  __device__ __forceinline__ uint32_t rkr(int, int i) const {
    return right ? kDpfKeys[1].rkr[i] : kDpfKeys[0].rkr[i];
  }
};
struct PairSelect {  // generic keys from a kernel argument
  const KeyPair& kp;
  bool right;
  __device__ __forceinline__ uint32_t rk(int, int i) const {
    return right ? kp.k[1].rk[i] : kp.k[0].rk[i];
  }
  __device__ __forceinline__ uint32_t rkr(int, int i) const {
    return right ? kp.k[1].rkr[i] : kp.k[0].rkr[i];
  }
};

// N independent AES-128 encryptions in lockstep.  Each round first forms all
// 16N table addresses (v_perm), then issues all 16N ds_read_b32 back to back
// (sched_group_barrier keeps the scheduler from splitting them into small
// waitcnt-separated groups), then combines: per output column
// T0[a] ^ T1[b] ^ rotl16(T0[c] ^ T1[d] ^ rotr16(rk)) = 2 v_bitop3 + 1 alignbit.
template <int N, class K>
__device__ __forceinline__ void AesN(uint32_t (&w)[N][4], const K& key,
                                     const Lds& L) {
#pragma unroll
  for (int n = 0; n < N; ++n)
#pragma unroll
    for (int c = 0; c < 4; ++c) w[n][c] ^= key.rk(n, c);
#pragma unroll
  for (int r = 1; r < 10; ++r) {
    uint32_t t[N][4][4];
#pragma unroll
    for (int n = 0; n < N; ++n)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        t[n][c][0] = LoadT0(L, w[n][c], 0);
        t[n][c][1] = LoadT1(L, w[n][(c + 1) & 3], 1);
        t[n][c][2] = LoadT0(L, w[n][(c + 2) & 3], 2);
        t[n][c][3] = LoadT1(L, w[n][(c + 3) & 3], 3);
      }
    __builtin_amdgcn_sched_group_barrier(0x002, 16 * N, 0);  // address VALU
    __builtin_amdgcn_sched_group_barrier(0x100, 16 * N, 0);  // DS reads
#pragma unroll
    for (int n = 0; n < N; ++n)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        w[n][c] = Xor3(t[n][c][0], t[n][c][1],
                       Rotl16(Xor3(t[n][c][2], t[n][c][3], key.rkr(n, 4 * r + c))));
  }
  // Last round: S-box bytes are byte 1/2 of T0 and byte 3 of T1.
  uint32_t t[N][4][4];
#pragma unroll
  for (int n = 0; n < N; ++n)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      t[n][c][0] = LoadT0(L, w[n][c], 0);
      t[n][c][1] = LoadT0(L, w[n][(c + 1) & 3], 1);
      t[n][c][2] = LoadT0(L, w[n][(c + 2) & 3], 2);
      t[n][c][3] = LoadT1(L, w[n][(c + 3) & 3], 3);
    }
  __builtin_amdgcn_sched_group_barrier(0x002, 16 * N, 0);
  __builtin_amdgcn_sched_group_barrier(0x100, 16 * N, 0);
#pragma unroll
  for (int n = 0; n < N; ++n)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint32_t lo = __builtin_amdgcn_perm(t[n][c][1], t[n][c][0], 0x0c0c0501u);
      const uint32_t hi = __builtin_amdgcn_perm(t[n][c][3], t[n][c][2], 0x07020c0cu);
      w[n][c] = Xor3(lo, hi, key.rk(n, 40 + c));
    }
}

// sigma(x) = (x.hi ^ x.lo, x.hi) (aes_128_fixed_key_hash.cc:75-78) in words.
__device__ __forceinline__ void Sigma(const uint32_t (&x)[4], uint32_t (&s)[4]) {
  s[0] = x[2];
  s[1] = x[3];
  s[2] = x[0] ^ x[2];
  s[3] = x[1] ^ x[3];
}

__device__ __forceinline__ u128 ToU128(const uint32_t (&x)[4]) {
  return (u128)x[0] | ((u128)x[1] << 32) | ((u128)x[2] << 64) | ((u128)x[3] << 96);
}
__device__ __forceinline__ void FromU128(u128 v, uint32_t (&x)[4]) {
  x[0] = (uint32_t)v;
  x[1] = (uint32_t)(v >> 32);
  x[2] = (uint32_t)(v >> 64);
  x[3] = (uint32_t)(v >> 96);
}

// ----------------------------------------------------------------------------
// Value conversion + correction (vth:216-328, 447-460, 507-515, 586-606;
// int_mod_n.h:121-250; h:852-858)
// ----------------------------------------------------------------------------

__device__ __forceinline__ u128 MaskBytes(int nbytes) {
  return nbytes >= 16 ? ~(u128)0 : (((u128)1 << (8 * nbytes)) - 1);
}

template <int BN>
__device__ __forceinline__ u128 PickWord(const u128 (&W)[BN], int j) {
  u128 r = W[0];
#pragma unroll
  for (int i = 1; i < BN; ++i)
    if (j == i) r = W[i];
  return r;
}

// Little-endian bytes [off, off + nbytes) of the hashed blocks.
template <int BN>
__device__ __forceinline__ u128 GetBytes(const u128 (&W)[BN], int off, int nbytes) {
  int j = off >> 4;
  int sh = (off & 15) * 8;
  u128 v = PickWord<BN>(W, j) >> sh;
  if (sh != 0 && j + 1 < BN) v |= PickWord<BN>(W, j + 1) << (128 - sh);
  return v & MaskBytes(nbytes);
}

__device__ __forceinline__ u128 ScAdd(const ScalarDev& s, u128 a, u128 b) {
  if (s.kind == DPF_AMD_KIND_INTEGER) return (a + b) & MaskBytes(s.bytes);
  if (s.kind == DPF_AMD_KIND_XOR_WRAPPER) return a ^ b;
  u128 x = s.mod - b;  // IntModN AddBaseInteger (int_mod_n.h:213-223)
  return a >= x ? a - x : s.mod - x + a;
}

__device__ __forceinline__ u128 ScNeg(const ScalarDev& s, u128 a) {
  if (s.kind == DPF_AMD_KIND_INTEGER) return (0 - a) & MaskBytes(s.bytes);
  if (s.kind == DPF_AMD_KIND_XOR_WRAPPER) return a;
  return a == 0 ? (u128)0 : s.mod - a;
}

// block -> (block / m, block % m).  Pseudo-Mersenne moduli m = 2^w - c with
// small c fold the high part (2^w = c mod m); others use 128-bit division.
__device__ __forceinline__ void DivMod(const ScalarDev& s, u128 x, u128& q, u128& r) {
  if (s.use_fold) {
    const int w = s.fold_w;
    const u128 low = ((u128)1 << w) - 1;
    u128 qq = 0;
    while ((x >> w) != 0) {
      u128 hi = x >> w;
      qq += hi;
      x = hi * s.fold_c + (x & low);
    }
    if (x >= s.mod) {
      x -= s.mod;
      qq += 1;
    }
    q = qq;
    r = x;
  } else {
    q = x / s.mod;
    r = x % s.mod;
  }
}

__device__ __forceinline__ void StoreScalar(char* p, int nbytes, u128 v) {
  switch (nbytes) {
    case 1:
      *reinterpret_cast<uint8_t*>(p) = (uint8_t)v;
      break;
    case 2:
      *reinterpret_cast<uint16_t*>(p) = (uint16_t)v;
      break;
    case 4:
      *reinterpret_cast<uint32_t*>(p) = (uint32_t)v;
      break;
    case 8:
      *reinterpret_cast<uint64_t*>(p) = (uint64_t)v;
      break;
    default: {
      uint4 u;
      u.x = (uint32_t)v;
      u.y = (uint32_t)(v >> 32);
      u.z = (uint32_t)(v >> 64);
      u.w = (uint32_t)(v >> 96);
      *reinterpret_cast<uint4*>(p) = u;
    }
  }
}

__device__ __forceinline__ u128 Correct(const ScalarDev& s, u128 v, bool t,
                                        u128 corr, int party) {
  if (t) v = ScAdd(s, v, corr);
  if (party == 1) v = ScNeg(s, v);
  return v;
}

// Converts the hashed blocks of one tree leaf and writes elements
// [e_begin, e_end) (ConvertBytesToArrayOf + correction, h:846-862).
// `corr` points at the correction of element 0; `elem_out(e)` gives the
// destination of element e.
template <int BN, class Out>
__device__ __forceinline__ void EmitLeaf(const VtDev& vt, const u128 (&W)[BN],
                                         bool t, int party, const u128* corr,
                                         int e_begin, int e_end, Out elem_out) {
  if (vt.direct) {
    for (int e = e_begin; e < e_end; ++e) {
      char* dst = elem_out(e);
      for (int s = 0; s < vt.ns; ++s) {
        const ScalarDev& sc = vt.sc[s];
        u128 v = GetBytes<BN>(W, e * vt.esz + sc.in_off, sc.bytes);
        v = Correct(sc, v, t, corr[e * vt.ns + s], party);
        StoreScalar(dst + sc.out_off, sc.bytes, v);
      }
    }
    return;
  }
  // Sampling path (an IntModN is present; epb == 1).
  char* dst = elem_out(0);
  u128 block = W[0];
  int pos = 16;
  for (int s = 0; s < vt.ns; ++s) {
    const ScalarDev& sc = vt.sc[s];
    const bool update = s + 1 < vt.ns;
    u128 v;
    if (sc.kind == DPF_AMD_KIND_INT_MOD_N) {
      u128 q, r;
      DivMod(sc, block, q, r);
      v = r;
      if (update) {
        block = (sc.bytes < 16) ? (q << (8 * sc.bytes)) : (u128)0;
        block |= GetBytes<BN>(W, pos, sc.bytes);
        pos += sc.bytes;
      }
    } else {
      v = block & MaskBytes(sc.bytes);
      if (update) {
        block = (sc.bytes < 16) ? (block & ~MaskBytes(sc.bytes)) : (u128)0;
        block |= GetBytes<BN>(W, pos, sc.bytes);
        pos += sc.bytes;
      }
    }
    v = Correct(sc, v, t, corr[s], party);
    StoreScalar(dst + sc.out_off, sc.bytes, v);
  }
}

// Value PRG of NS seeds: block j of seed n = H_value(seed_n + j)
// (HashExpandedSeeds, cc:523-547).
template <int NS, int BN>
__device__ __forceinline__ void HashSeeds(const uint32_t (&x)[NS][4], u128 (&W)[NS][BN],
                                          const Lds& L) {
  uint32_t st[NS * BN][4], sg[NS * BN][4];
#pragma unroll
  for (int n = 0; n < NS; ++n) {
    u128 base = ToU128(x[n]);
#pragma unroll
    for (int j = 0; j < BN; ++j) {
      uint32_t y[4];
      FromU128(base + (u128)j, y);
      Sigma(y, sg[n * BN + j]);
#pragma unroll
      for (int c = 0; c < 4; ++c) st[n * BN + j][c] = sg[n * BN + j][c];
    }
  }
  AesN<NS * BN>(st, DpfKeyAt<2>{}, L);
#pragma unroll
  for (int i = 0; i < NS * BN; ++i) {
#pragma unroll
    for (int c = 0; c < 4; ++c) st[i][c] ^= sg[i][c];
  }
#pragma unroll
  for (int n = 0; n < NS; ++n)
#pragma unroll
    for (int j = 0; j < BN; ++j) W[n][j] = ToU128(st[n * BN + j]);
}

// ----------------------------------------------------------------------------
// Tree steps (ExpandSeeds cc:327-370; EvaluateSeeds evaluate_prg_hwy.cc:
// 552-634).  Seed correction is applied before the control bit is extracted.
// ----------------------------------------------------------------------------

struct Cw {
  uint32_t seed[4];
  uint32_t cl, cr;
};

__device__ __forceinline__ Cw LoadCw(const uint4* cw_seed, const uint8_t* ccl,
                                     const uint8_t* ccr, int64_t i) {
  uint4 s = cw_seed[i];
  Cw c;
  c.seed[0] = s.x;
  c.seed[1] = s.y;
  c.seed[2] = s.z;
  c.seed[3] = s.w;
  c.cl = ccl[i];
  c.cr = ccr[i];
  return c;
}

// Both children of x (left at 2j, right at 2j+1).
__device__ __forceinline__ void Expand2(const uint32_t (&x)[4], uint32_t t, const Cw& cw,
                                        const Lds& L, uint32_t (&l)[4], uint32_t& tl,
                                        uint32_t (&r)[4], uint32_t& tr) {
  uint32_t s[4], st[2][4];
  Sigma(x, s);
#pragma unroll
  for (int c = 0; c < 4; ++c) st[0][c] = st[1][c] = s[c];
  AesN<2>(st, DpfLeftRight{}, L);
  const uint32_t m = 0u - t;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    l[c] = st[0][c] ^ s[c] ^ (cw.seed[c] & m);
    r[c] = st[1][c] ^ s[c] ^ (cw.seed[c] & m);
  }
  tl = (l[0] & 1u) ^ (t & cw.cl);
  tr = (r[0] & 1u) ^ (t & cw.cr);
  l[0] &= ~1u;
  r[0] &= ~1u;
}

// One path step with the key chosen by `bit` (per lane).
template <class K>
__device__ __forceinline__ void WalkStep(uint32_t (&x)[4], uint32_t& t, uint32_t bit,
                                         const Cw& cw, const K& key, const Lds& L) {
  uint32_t s[4], st[1][4];
  Sigma(x, s);
#pragma unroll
  for (int c = 0; c < 4; ++c) st[0][c] = s[c];
  AesN<1>(st, key, L);
  const uint32_t m = 0u - t;
#pragma unroll
  for (int c = 0; c < 4; ++c) x[c] = st[0][c] ^ s[c] ^ (cw.seed[c] & m);
  uint32_t nt = (x[0] & 1u) ^ (t & (bit ? cw.cr : cw.cl));
  x[0] &= ~1u;
  t = nt;
}

// ----------------------------------------------------------------------------
// Leaf emitters: value conversion + correction + store of one tree leaf.
// EmitGeneric handles every supported T through the runtime descriptor; the
// specialised emitters cover the benchmark types without 128-bit generic code
// (they produce bit-identical results; tests compare both against the oracle).
// ----------------------------------------------------------------------------

struct ExpandArgs {
  const uint4* root_seeds;
  const uint8_t* root_cb;
  const uint4* cw_seed;
  const uint8_t* ccl;
  const uint8_t* ccr;
  char* out;
  int64_t chunk_begin;
  int64_t chunk_end;
  int64_t leaf_begin;
  int64_t leaf_end;
  int32_t walk;  // levels walked per thread before the DFS
  int32_t pad;
};

struct ExpandCtx {
  const ExpandArgs& a;
  const VtDev& vt;
  const Lds& L;
};

// Value PRG of one seed: block j = H_value(seed + j) (cc:523-547).
template <int NS, int BN>
__device__ __forceinline__ void HashWords(const uint32_t (&x)[NS][4],
                                          uint32_t (&h)[NS][BN][4], const Lds& L) {
  uint32_t st[NS * BN][4], sg[NS * BN][4];
#pragma unroll
  for (int n = 0; n < NS; ++n) {
#pragma unroll
    for (int j = 0; j < BN; ++j) {
      uint32_t y[4];
      if (j == 0) {
#pragma unroll
        for (int c = 0; c < 4; ++c) y[c] = x[n][c];
      } else {
        FromU128(ToU128(x[n]) + (u128)j, y);
      }
      Sigma(y, sg[n * BN + j]);
#pragma unroll
      for (int c = 0; c < 4; ++c) st[n * BN + j][c] = sg[n * BN + j][c];
    }
  }
  AesN<NS * BN>(st, DpfKeyAt<2>{}, L);
#pragma unroll
  for (int n = 0; n < NS; ++n)
#pragma unroll
    for (int j = 0; j < BN; ++j)
#pragma unroll
      for (int c = 0; c < 4; ++c) h[n][j][c] = st[n * BN + j][c] ^ sg[n * BN + j][c];
}

template <int BN>
struct EmitGeneric {
  static constexpr int kBN = BN;
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
template <int B>
struct EmitDirect {
  static constexpr int kBN = 1;
  __device__ static void Emit(const ExpandCtx& E, const uint32_t (&h)[1][4], uint32_t t,
                              int64_t g) {
    const VtDev& vt = E.vt;
    if (g < E.a.leaf_begin || g >= E.a.leaf_end) return;
    uint32_t w[4], c[4];
    const uint32_t m = 0u - t;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      w[i] = h[0][i];
      c[i] = (uint32_t)(vt.corr_packed >> (32 * i)) & m;
    }
    if (vt.sc[0].kind == DPF_AMD_KIND_XOR_WRAPPER) {
#pragma unroll
      for (int i = 0; i < 4; ++i) w[i] ^= c[i];
    } else {
      SwarAdd<B>(w, c);
      if (vt.party == 1) SwarNeg<B>(w);
    }
    char* dst = E.a.out + (g - E.a.leaf_begin) * (int64_t)vt.cepb * B;
    if (vt.cepb * B == 16) {
      *reinterpret_cast<uint4*>(dst) = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
      const u128 v = ToU128(w);
      for (int e = 0; e < vt.cepb; ++e) StoreScalar(dst + e * B, B, v >> (8 * B * e));
    }
  }
};

// T = Tuple<uint32_t, IntModN<uint64_t, m>> with m = 2^64 - c, c < 2^56
// (the c5 benchmark type).  Sampling path of vth:230-251, 303-328, 447-460:
// element 0 = low 32 bits of block 0; block := (block & ~0xffffffff) |
// bytes[16..20); element 1 = block mod m.
struct EmitU32ModN64 {
  static constexpr int kBN = 2;
  __device__ static void Emit(const ExpandCtx& E, const uint32_t (&h)[2][4], uint32_t t,
                              int64_t g) {
    const VtDev& vt = E.vt;
    if (g < E.a.leaf_begin || g >= E.a.leaf_end) return;
    uint32_t v0 = h[0][0];
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
    uint64_t v1 = xlo >= mod ? xlo - mod : xlo;
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
    char* dst = E.a.out + (g - E.a.leaf_begin) * (int64_t)vt.stride;
    if (vt.sc[0].out_off == 8 && vt.sc[1].out_off == 0 && vt.stride == 16) {
      *reinterpret_cast<uint4*>(dst) = make_uint4((uint32_t)v1, (uint32_t)(v1 >> 32), v0, 0u);
    } else {
      *reinterpret_cast<uint32_t*>(dst + vt.sc[0].out_off) = v0;
      *reinterpret_cast<uint64_t*>(dst + vt.sc[1].out_off) = v1;
    }
  }
};

// ----------------------------------------------------------------------------
// Fused subtree expansion kernel: each thread walks from its root to the root
// of a 2^D-leaf subtree (both children computed, the path child kept), then
// expands it depth-first in registers (right children kept per level), hashes
// and emits every leaf.
// ----------------------------------------------------------------------------

template <int DEPTH, class Em>
__device__ __forceinline__ void Dfs(const ExpandCtx& E, const uint32_t (&x)[4], uint32_t t,
                                    int level, int64_t leaf) {
  constexpr int BN = Em::kBN;
  if constexpr (DEPTH == 0) {
    uint32_t xs[1][4] = {{x[0], x[1], x[2], x[3]}};
    uint32_t h[1][BN][4];
    HashWords<1, BN>(xs, h, E.L);
    Em::Emit(E, h[0], t, leaf);
  } else {
    const Cw cw = LoadCw(E.a.cw_seed, E.a.ccl, E.a.ccr, level);
    uint32_t l[4], r[4], tl, tr;
    Expand2(x, t, cw, E.L, l, tl, r, tr);
    if constexpr (DEPTH == 1 && BN == 1) {
      uint32_t xs[2][4] = {{l[0], l[1], l[2], l[3]}, {r[0], r[1], r[2], r[3]}};
      uint32_t h[2][1][4];
      HashWords<2, 1>(xs, h, E.L);
      Em::Emit(E, h[0], tl, 2 * leaf);
      Em::Emit(E, h[1], tr, 2 * leaf + 1);
    } else {
#pragma unroll 1
      for (int b = 0; b < 2; ++b) {
        uint32_t y[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) y[c] = b ? r[c] : l[c];
        Dfs<DEPTH - 1, Em>(E, y, b ? tr : tl, level + 1, 2 * leaf + b);
      }
    }
  }
}

template <int D, class Em>
__global__ __launch_bounds__(kBlock, 2) void KExpand(ExpandArgs a, VtDev vt) {
  __shared__ uint32_t tab[kTabWords];
  FillTables(tab);
  __syncthreads();
  const Lds L = MakeLds(tab);
  const ExpandCtx E{a, vt, L};
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t chunk = a.chunk_begin + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
       chunk < a.chunk_end; chunk += stride) {
    const int64_t root = chunk >> a.walk;
    const uint64_t path = (uint64_t)chunk & ((a.walk >= 63) ? ~0ull : ((1ull << a.walk) - 1));
    uint4 s = a.root_seeds[root];
    uint32_t x[4] = {s.x, s.y, s.z, s.w};
    uint32_t t = a.root_cb[root];
    for (int i = 0; i < a.walk; ++i) {
      const uint32_t bit = (uint32_t)(path >> (a.walk - 1 - i)) & 1u;
      const Cw cw = LoadCw(a.cw_seed, a.ccl, a.ccr, i);
      uint32_t l[4], r[4], tl, tr;
      Expand2(x, t, cw, L, l, tl, r, tr);
#pragma unroll
      for (int c = 0; c < 4; ++c) x[c] = bit ? r[c] : l[c];
      t = bit ? tr : tl;
    }
    Dfs<D, Em>(E, x, t, a.walk, chunk);
  }
}

// ----------------------------------------------------------------------------
// Path-walk kernels
// ----------------------------------------------------------------------------

struct WalkArgs {
  int64_t num_seeds;
  int64_t num_cw;
  const uint4* seeds_in;
  const uint8_t* cb_in;
  const uint4* paths;
  const uint4* cw_seed;
  const uint8_t* ccl;
  const uint8_t* ccr;
  uint4* seeds_out;
  uint8_t* cb_out;
  int32_t num_levels;
  int32_t rightshift;
};

__device__ __forceinline__ uint32_t PathBit(const uint4& p, int bit_index) {
  if (bit_index >= 128) return 0;
  uint32_t w = bit_index < 32 ? p.x : bit_index < 64 ? p.y : bit_index < 96 ? p.z : p.w;
  return (w >> (bit_index & 31)) & 1u;
}

// Generic-key EvaluateSeeds (evaluate_prg_hwy.cc:552-634).
__global__ __launch_bounds__(kBlock, 2) void KEvaluateSeeds(WalkArgs a, KeyPair kp) {
  __shared__ uint32_t tab[kTabWords];
  FillTables(tab);
  __syncthreads();
  const Lds L = MakeLds(tab);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.num_seeds;
       i += stride) {
    uint4 s = a.seeds_in[i];
    uint32_t x[4] = {s.x, s.y, s.z, s.w};
    uint32_t t = a.cb_in[i];
    const uint4 p = a.paths[i];
    const bool per_seed = a.num_cw > a.num_levels;
    for (int level = 0; level < a.num_levels; ++level) {
      const uint32_t bit = PathBit(p, a.num_levels - level - 1 + a.rightshift);
      const int64_t ci = per_seed ? (int64_t)level * a.num_seeds + i : level;
      const Cw cw = LoadCw(a.cw_seed, a.ccl, a.ccr, ci);
      WalkStep(x, t, bit, cw, PairSelect{kp, bit != 0}, L);
    }
    a.seeds_out[i] = make_uint4(x[0], x[1], x[2], x[3]);
    a.cb_out[i] = (uint8_t)t;
  }
}

struct PointsArgs {
  WalkArgs w;
  const uint8_t* block_index;
  const int8_t* party;
  const uint4* value_corrections;  // per seed: epb * ns 128-bit words
  char* out;
};

// EvaluateAtImpl / EvaluateAndApply per-point evaluation (h:1013-1063,
// 1143-1189).
template <int BN>
__global__ __launch_bounds__(kBlock, 2) void KEvaluatePoints(PointsArgs a, VtDev vt) {
  __shared__ uint32_t tab[kTabWords];
  FillTables(tab);
  __syncthreads();
  const Lds L = MakeLds(tab);
  const WalkArgs& w = a.w;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int per_elem = vt.epb * vt.ns;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < w.num_seeds;
       i += stride) {
    uint4 s = w.seeds_in[i];
    uint32_t x[1][4] = {{s.x, s.y, s.z, s.w}};
    uint32_t t = w.cb_in[i];
    const uint4 p = w.paths[i];
    const bool per_seed = w.num_cw > w.num_levels;
    for (int level = 0; level < w.num_levels; ++level) {
      const uint32_t bit = PathBit(p, w.num_levels - level - 1 + w.rightshift);
      const int64_t ci = per_seed ? (int64_t)level * w.num_seeds + i : level;
      const Cw cw = LoadCw(w.cw_seed, w.ccl, w.ccr, ci);
      WalkStep(x[0], t, bit, cw, DpfSelect{bit != 0}, L);
    }
    if (w.seeds_out) {
      w.seeds_out[i] = make_uint4(x[0][0], x[0][1], x[0][2], x[0][3]);
      w.cb_out[i] = (uint8_t)t;
    }
    u128 W[1][BN];
    HashSeeds<1, BN>(x, W, L);
    const int bi = a.block_index ? a.block_index[i] : 0;
    const int party = a.party ? a.party[i] : vt.party;
    char* dst = a.out + i * (int64_t)vt.stride;
    if (a.value_corrections) {
      u128 corr[kMaxCorrections];
      const uint4* src = a.value_corrections + i * per_elem;
      for (int j = 0; j < per_elem; ++j) {
        uint4 c = src[j];
        corr[j] = (u128)c.x | ((u128)c.y << 32) | ((u128)c.z << 64) | ((u128)c.w << 96);
      }
      EmitLeaf<BN>(vt, W[0], t != 0, party, corr, bi, bi + 1,
                   [dst](int) { return dst; });
    } else {
      EmitLeaf<BN>(vt, W[0], t != 0, party, vt.corr, bi, bi + 1,
                   [dst](int) { return dst; });
    }
  }
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
    AesN<1>(st, PairSelect{kp, false}, L);
    out[i] = make_uint4(st[0][0] ^ s[0], st[0][1] ^ s[1], st[0][2] ^ s[2], st[0][3] ^ s[3]);
  }
}

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
constexpr int kFoldWords = 4;
constexpr int kFoldSlices = 64;

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

constexpr int kScanBlock = 256;
constexpr int kScanWaves = kScanBlock / 64;
constexpr int kScanUnroll = 8;

struct ScanArgs {
  const uint4* db;
  const uint4* sel;     // [query][selection_blocks]
  uint4* partials;      // [blockIdx.x][query][C]
  int64_t num_records;
  int64_t sel_blocks;
  int32_t C;            // 16-byte chunks per record
  int32_t q0;           // first query of this pass
  int32_t nq;           // queries in this pass (<= QN)
  int32_t total_q;
};

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

// ----------------------------------------------------------------------------
// Host side (Tier-1 C ABI)
// ----------------------------------------------------------------------------

namespace {

int HipCheck(hipError_t e, const char* what) {
  if (e == hipSuccess) return DPF_AMD_OK;
  const int code =
      (e == hipErrorOutOfMemory) ? DPF_AMD_RESOURCE_EXHAUSTED : DPF_AMD_INTERNAL;
  return SetError(code, std::string(what) + ": " + hipGetErrorString(e));
}

int LaunchCheck(const char* what) { return HipCheck(hipGetLastError(), what); }

int GridFor(int64_t items, int block, int max_blocks) {
  int64_t g = (items + block - 1) / block;
  if (g < 1) g = 1;
  if (g > max_blocks) g = max_blocks;
  return (int)g;
}

KeyPair MakeKeyPair(uint64_t l_lo, uint64_t l_hi, uint64_t r_lo, uint64_t r_hi) {
  KeyPair kp;
  kp.k[0] = ExpandAesKey(l_lo, l_hi);
  kp.k[1] = ExpandAesKey(r_lo, r_hi);
  return kp;
}

int BnTemplate(int bn) {
  if (bn <= 1) return 1;
  if (bn == 2) return 2;
  return 4;
}

template <int D, class Em>
int LaunchExpand(int grid, hipStream_t st, const ExpandArgs& a, const VtDev& vt) {
  hipLaunchKernelGGL((KExpand<D, Em>), dim3(grid), dim3(kBlock), 0, st, a, vt);
  return LaunchCheck("expand kernel launch");
}

template <class Em>
int LaunchExpandAnyD(int D, int grid, hipStream_t st, const ExpandArgs& a, const VtDev& vt) {
  switch (D) {
    case 0:
      return LaunchExpand<0, Em>(grid, st, a, vt);
    case 1:
      return LaunchExpand<1, Em>(grid, st, a, vt);
    case 2:
      return LaunchExpand<2, Em>(grid, st, a, vt);
    case 4:
      return LaunchExpand<4, Em>(grid, st, a, vt);
    default:
      return LaunchExpand<8, Em>(grid, st, a, vt);
  }
}

// Picks the emitter for the value type.
int LaunchExpandForType(int D, int grid, hipStream_t st, const ExpandArgs& a,
                        const VtDev& vt) {
  const bool single_direct = vt.direct && vt.ns == 1 && vt.sc[0].in_off == 0 &&
                             vt.sc[0].out_off == 0 && vt.stride == vt.sc[0].bytes &&
                             vt.bn == 1 && vt.epb * vt.sc[0].bytes == 16;
  if (single_direct) {
    switch (vt.sc[0].bytes) {
      case 1:
        return LaunchExpandAnyD<EmitDirect<1>>(D, grid, st, a, vt);
      case 2:
        return LaunchExpandAnyD<EmitDirect<2>>(D, grid, st, a, vt);
      case 4:
        return LaunchExpandAnyD<EmitDirect<4>>(D, grid, st, a, vt);
      case 8:
        return LaunchExpandAnyD<EmitDirect<8>>(D, grid, st, a, vt);
      default:
        return LaunchExpandAnyD<EmitDirect<16>>(D, grid, st, a, vt);
    }
  }
  const bool u32_modn64 =
      !vt.direct && vt.ns == 2 && vt.bn == 2 && vt.epb == 1 &&
      vt.sc[0].kind == DPF_AMD_KIND_INTEGER && vt.sc[0].bytes == 4 &&
      vt.sc[1].kind == DPF_AMD_KIND_INT_MOD_N && vt.sc[1].bytes == 8 &&
      vt.sc[1].use_fold && vt.sc[1].fold_w == 64 && (vt.sc[1].fold_c >> 56) == 0;
  if (u32_modn64) return LaunchExpandAnyD<EmitU32ModN64>(D, grid, st, a, vt);
  switch (BnTemplate(vt.bn)) {
    case 1:
      return LaunchExpandAnyD<EmitGeneric<1>>(D, grid, st, a, vt);
    case 2:
      return LaunchExpandAnyD<EmitGeneric<2>>(D, grid, st, a, vt);
    default:
      return LaunchExpandAnyD<EmitGeneric<4>>(D, grid, st, a, vt);
  }
}

}  // namespace

int MakeVtDev(const dpf_amd_value_type& vt, const uint64_t* correction, int party,
              int cepb, VtDev* out) {
  std::memset(out, 0, sizeof(*out));
  if (vt.num_scalars <= 0 || vt.num_scalars > kMaxScalars)
    return SetError(DPF_AMD_UNIMPLEMENTED, "unsupported number of tuple elements");
  if (vt.elements_per_block * vt.num_scalars > kMaxCorrections)
    return SetError(DPF_AMD_UNIMPLEMENTED, "too many packed elements");
  if (vt.blocks_needed < 1 || vt.blocks_needed > DPF_AMD_MAX_BLOCKS_NEEDED)
    return SetError(DPF_AMD_UNIMPLEMENTED, "blocks_needed out of supported range");
  if (cepb < 1 || cepb > vt.elements_per_block)
    return SetError(DPF_AMD_INVALID_ARGUMENT, "bad corrected_elements_per_block");
  out->ns = vt.num_scalars;
  out->direct = vt.directly_convertible;
  out->epb = vt.elements_per_block;
  out->esz = vt.element_size;
  out->bn = vt.blocks_needed;
  out->stride = vt.out_stride;
  out->cepb = cepb;
  out->party = party;
  for (int s = 0; s < vt.num_scalars; ++s) {
    const dpf_amd_scalar& in = vt.scalars[s];
    ScalarDev& d = out->sc[s];
    d.kind = in.kind;
    d.bytes = in.bytes;
    d.in_off = in.in_offset;
    d.out_off = in.out_offset;
    d.mod = (u128)in.modulus[0] | ((u128)in.modulus[1] << 64);
    d.use_fold = 0;
    if (in.kind == DPF_AMD_KIND_INT_MOD_N) {
      if (d.mod == 0) return SetError(DPF_AMD_INVALID_ARGUMENT, "IntModN modulus is 0");
      // w = bit length of (m - 1): m = 2^w - c with 0 <= c < 2^(w-1).
      u128 mm = d.mod - 1;
      int w = 0;
      while (w < 128 && (mm >> w) != 0) ++w;
      if (w >= 1 && w <= 127) {
        u128 c = ((u128)1 << w) - d.mod;
        if (w >= 8 && (c >> (w - 8)) == 0) {
          d.use_fold = 1;
          d.fold_w = w;
          d.fold_c = c;
        }
      }
    }
  }
  if (correction) {
    for (int j = 0; j < vt.elements_per_block * vt.num_scalars; ++j)
      out->corr[j] = (u128)correction[2 * j] | ((u128)correction[2 * j + 1] << 64);
  }
  out->corr_packed = 0;
  if (vt.num_scalars == 1 && vt.scalars[0].bytes * vt.elements_per_block <= 16) {
    const int b = vt.scalars[0].bytes;
    for (int e = 0; e < vt.elements_per_block; ++e)
      out->corr_packed |= (out->corr[e] & (b >= 16 ? ~(u128)0 : (((u128)1 << (8 * b)) - 1)))
                          << (8 * b * e);
  }
  return DPF_AMD_OK;
}

}  // namespace dpf_amd

using namespace dpf_amd;

extern "C" {

const char* dpf_amd_version(void) { return "dpf_amd 0.1 (gfx950, T-table AES in LDS)"; }

int dpf_amd_device_count(int* count) {
  return HipCheck(hipGetDeviceCount(count), "hipGetDeviceCount");
}

int dpf_amd_aes128_mmo(uint64_t key_lo, uint64_t key_hi, const void* in, void* out,
                       int64_t n, void* stream) {
  if (n < 0) return SetError(DPF_AMD_INVALID_ARGUMENT, "negative size");
  if (n == 0) return DPF_AMD_OK;
  if (!in || !out) return SetError(DPF_AMD_INVALID_ARGUMENT, "null buffer");
  KeyPair kp = MakeKeyPair(key_lo, key_hi, key_lo, key_hi);
  hipLaunchKernelGGL(KAesMmo, dim3(GridFor(n, kBlock, 2048)), dim3(kBlock), 0,
                     (hipStream_t)stream, (const uint4*)in, (uint4*)out, n, kp);
  return LaunchCheck("aes kernel launch");
}

int dpf_amd_evaluate_seeds(int64_t num_seeds, int num_levels, int64_t num_correction_words,
                           const void* seeds_in, const uint8_t* control_bits_in,
                           const void* paths, int paths_rightshift,
                           const void* correction_seeds, const uint8_t* ccl,
                           const uint8_t* ccr, uint64_t key_left_lo, uint64_t key_left_hi,
                           uint64_t key_right_lo, uint64_t key_right_hi, void* seeds_out,
                           uint8_t* control_bits_out, void* stream) {
  if (num_correction_words != num_levels &&
      num_correction_words != (int64_t)num_levels * num_seeds)
    return SetError(DPF_AMD_INVALID_ARGUMENT,
                    "`num_correction_words` must be equal to `num_levels` or "
                    "`num_levels * num_seeds`");
  if (num_seeds < 0 || num_levels < 0 || paths_rightshift < 0)
    return SetError(DPF_AMD_INVALID_ARGUMENT, "negative size");
  if (num_seeds == 0) return DPF_AMD_OK;
  if (num_levels == 0) {
    hipStream_t st = (hipStream_t)stream;
    int rc = DPF_AMD_OK;
    if (seeds_out != seeds_in)
      rc = HipCheck(hipMemcpyAsync(seeds_out, seeds_in, 16 * num_seeds,
                                   hipMemcpyDeviceToDevice, st), "copy");
    if (rc == DPF_AMD_OK && control_bits_out != control_bits_in)
      rc = HipCheck(hipMemcpyAsync(control_bits_out, control_bits_in, num_seeds,
                                   hipMemcpyDeviceToDevice, st), "copy");
    return rc;
  }
  WalkArgs a;
  a.num_seeds = num_seeds;
  a.num_cw = num_correction_words;
  a.seeds_in = (const uint4*)seeds_in;
  a.cb_in = control_bits_in;
  a.paths = (const uint4*)paths;
  a.cw_seed = (const uint4*)correction_seeds;
  a.ccl = ccl;
  a.ccr = ccr;
  a.seeds_out = (uint4*)seeds_out;
  a.cb_out = control_bits_out;
  a.num_levels = num_levels;
  a.rightshift = paths_rightshift;
  KeyPair kp = MakeKeyPair(key_left_lo, key_left_hi, key_right_lo, key_right_hi);
  hipLaunchKernelGGL(KEvaluateSeeds, dim3(GridFor(num_seeds, kBlock, 4096)), dim3(kBlock), 0,
                     (hipStream_t)stream, a, kp);
  return LaunchCheck("evaluate_seeds kernel launch");
}

int dpf_amd_expand_and_correct(int64_t num_roots, const void* root_seeds,
                               const uint8_t* root_control_bits, int num_levels,
                               const void* correction_seeds, const uint8_t* ccl,
                               const uint8_t* ccr, const dpf_amd_value_type* vt,
                               const uint64_t* value_correction, int party,
                               int corrected_elements_per_block, int64_t leaf_begin,
                               int64_t leaf_end, void* out, void* stream) {
  if (num_levels < 0 || num_levels > 62)
    return SetError(DPF_AMD_INVALID_ARGUMENT,
                    "Trying to expand more than 62 tree levels at once. Please insert "
                    "intermediate hierarchy levels, or evaluate fewer hierarchy levels "
                    "at once.");
  if (num_roots < 0 || !vt) return SetError(DPF_AMD_INVALID_ARGUMENT, "bad arguments");
  if (num_roots > 0 && (num_roots > (INT64_MAX >> num_levels)))
    return SetError(DPF_AMD_INVALID_ARGUMENT, "Output size would be larger than 2**62.");
  const int64_t total_leaves = num_roots << num_levels;
  if (leaf_begin < 0 || leaf_end > total_leaves || leaf_begin > leaf_end)
    return SetError(DPF_AMD_INVALID_ARGUMENT, "leaf range out of bounds");
  if (leaf_begin == leaf_end) return DPF_AMD_OK;
  VtDev dev;
  int rc = MakeVtDev(*vt, value_correction, party, corrected_elements_per_block, &dev);
  if (rc != DPF_AMD_OK) return rc;
  // DFS depth D (compile-time); the upper num_levels - D levels are walked
  // per thread (1 AES/level), amortised over 2^D leaves.
  int D;
  if (num_levels >= 8)
    D = 8;
  else if (num_levels >= 4)
    D = 4;
  else if (num_levels >= 2)
    D = 2;
  else
    D = num_levels;
  // For small problems prefer more threads over deep DFS.
  while (D > 2 && ((leaf_end - leaf_begin) >> D) < 65536) D = (D == 8) ? 4 : 2;
  ExpandArgs a;
  a.root_seeds = (const uint4*)root_seeds;
  a.root_cb = root_control_bits;
  a.cw_seed = (const uint4*)correction_seeds;
  a.ccl = ccl;
  a.ccr = ccr;
  a.out = (char*)out;
  a.walk = num_levels - D;
  a.pad = 0;
  a.chunk_begin = leaf_begin >> D;
  a.chunk_end = (leaf_end + (1ll << D) - 1) >> D;
  a.leaf_begin = leaf_begin;
  a.leaf_end = leaf_end;
  const int grid = GridFor(a.chunk_end - a.chunk_begin, kBlock, 8192);
  return LaunchExpandForType(D, grid, (hipStream_t)stream, a, dev);
}

int dpf_amd_evaluate_points(int64_t num_seeds, const void* seeds, const uint8_t* control_bits,
                            const void* paths, int paths_rightshift, int num_levels,
                            int64_t num_correction_words, const void* correction_seeds,
                            const uint8_t* ccl, const uint8_t* ccr,
                            const dpf_amd_value_type* vt, const uint8_t* block_index,
                            const int8_t* party, int party_all,
                            const void* value_corrections,
                            const uint64_t* value_correction_all, void* out,
                            void* seeds_out, uint8_t* control_bits_out, void* stream) {
  if (num_correction_words != num_levels &&
      num_correction_words != (int64_t)num_levels * num_seeds)
    return SetError(DPF_AMD_INVALID_ARGUMENT,
                    "`num_correction_words` must be equal to `num_levels` or "
                    "`num_levels * num_seeds`");
  if (num_seeds < 0 || num_levels < 0 || !vt)
    return SetError(DPF_AMD_INVALID_ARGUMENT, "bad arguments");
  if (num_seeds == 0) return DPF_AMD_OK;
  VtDev dev;
  int rc = MakeVtDev(*vt, value_correction_all, party_all, vt->elements_per_block, &dev);
  if (rc != DPF_AMD_OK) return rc;
  PointsArgs a;
  a.w.num_seeds = num_seeds;
  a.w.num_cw = num_correction_words;
  a.w.seeds_in = (const uint4*)seeds;
  a.w.cb_in = control_bits;
  a.w.paths = (const uint4*)paths;
  a.w.cw_seed = (const uint4*)correction_seeds;
  a.w.ccl = ccl;
  a.w.ccr = ccr;
  a.w.seeds_out = (uint4*)seeds_out;
  a.w.cb_out = control_bits_out;
  a.w.num_levels = num_levels;
  a.w.rightshift = paths_rightshift;
  a.block_index = block_index;
  a.party = party;
  a.value_corrections = (const uint4*)value_corrections;
  a.out = (char*)out;
  const int grid = GridFor(num_seeds, kBlock, 4096);
  hipStream_t st = (hipStream_t)stream;
  switch (BnTemplate(dev.bn)) {
    case 1:
      hipLaunchKernelGGL((KEvaluatePoints<1>), dim3(grid), dim3(kBlock), 0, st, a, dev);
      break;
    case 2:
      hipLaunchKernelGGL((KEvaluatePoints<2>), dim3(grid), dim3(kBlock), 0, st, a, dev);
      break;
    default:
      hipLaunchKernelGGL((KEvaluatePoints<4>), dim3(grid), dim3(kBlock), 0, st, a, dev);
  }
  return LaunchCheck("evaluate_points kernel launch");
}

int dpf_amd_gather_rows(int64_t num_prefixes, const int64_t* src_offset,
                        int64_t outputs_per_prefix, int64_t stride, const void* in, void* out,
                        void* stream) {
  if (num_prefixes <= 0 || outputs_per_prefix <= 0) return DPF_AMD_OK;
  const int64_t total = num_prefixes * outputs_per_prefix * stride;
  hipLaunchKernelGGL(KGatherRows, dim3(GridFor(total, 256, 8192)), dim3(256), 0,
                     (hipStream_t)stream, num_prefixes, src_offset, outputs_per_prefix,
                     stride, (const char*)in, (char*)out);
  return LaunchCheck("gather kernel launch");
}

int dpf_amd_xor_fold(const void* parts, int num_parts, int64_t bytes, void* out,
                     void* stream) {
  if (num_parts <= 0 || bytes <= 0) return DPF_AMD_OK;
  hipStream_t st = (hipStream_t)stream;
  if (bytes % 16 == 0 && ((uintptr_t)parts % 16 == 0) && ((uintptr_t)out % 16 == 0)) {
    const int64_t words = bytes / 16;
    const int64_t blocks = (words + kFoldWords - 1) / kFoldWords;
    if (blocks > INT32_MAX) return SetError(DPF_AMD_INVALID_ARGUMENT, "xor fold too large");
    hipLaunchKernelGGL(KXorFold, dim3((unsigned)blocks), dim3(256), 0, st,
                       (const uint4*)parts, num_parts, words, (uint4*)out);
  } else {
    hipLaunchKernelGGL(KXorFoldBytes, dim3(GridFor(bytes, 256, 4096)), dim3(256), 0, st,
                       (const uint8_t*)parts, num_parts, bytes, (uint8_t*)out);
  }
  return LaunchCheck("xor fold kernel launch");
}

static int ScanGrid(int64_t num_records) {
  // ~8 resident 256-thread blocks per CU on 256 CUs; at least one tile per wave.
  const int64_t tiles = (num_records + 127) / 128;
  int64_t g = (tiles + kScanWaves - 1) / kScanWaves;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, 2048));
}

int64_t dpf_amd_inner_product_workspace_size(int64_t num_records, int64_t record_stride,
                                             int num_queries) {
  return (int64_t)ScanGrid(num_records) * num_queries * record_stride;
}

int dpf_amd_inner_product(const void* db, int64_t num_records, int64_t record_stride,
                          const void* selections, int64_t selection_blocks, int num_queries,
                          void* workspace, void* out, void* stream) {
  if (num_queries == 0) return DPF_AMD_OK;
  if (num_records < 0 || num_queries < 0)
    return SetError(DPF_AMD_INVALID_ARGUMENT, "negative size");
  if (record_stride <= 0 || record_stride % 16 != 0)
    return SetError(DPF_AMD_INVALID_ARGUMENT, "record_stride must be a positive multiple of 16");
  if (selection_blocks * 128 < num_records)
    return SetError(DPF_AMD_INVALID_ARGUMENT,
                    "`selections[0]` contains insufficient number of bits: " +
                        std::to_string(selection_blocks * 128) +
                        ", expected: " + std::to_string(num_records));
  hipStream_t st = (hipStream_t)stream;
  const int grid = ScanGrid(num_records);
  const int C = (int)(record_stride / 16);
  ScanArgs a;
  a.db = (const uint4*)db;
  a.sel = (const uint4*)selections;
  a.partials = (uint4*)workspace;
  a.num_records = num_records;
  a.sel_blocks = selection_blocks;
  a.C = C;
  a.total_q = num_queries;
  const dim3 g(grid, (C + 63) / 64);
  for (int q0 = 0; q0 < num_queries; q0 += 8) {
    const int nq = std::min(8, num_queries - q0);
    a.q0 = q0;
    a.nq = nq;
    if (nq == 1)
      hipLaunchKernelGGL((KPirScan<1>), g, dim3(kScanBlock), 0, st, a);
    else if (nq <= 2)
      hipLaunchKernelGGL((KPirScan<2>), g, dim3(kScanBlock), 0, st, a);
    else if (nq <= 4)
      hipLaunchKernelGGL((KPirScan<4>), g, dim3(kScanBlock), 0, st, a);
    else
      hipLaunchKernelGGL((KPirScan<8>), g, dim3(kScanBlock), 0, st, a);
    int rc = LaunchCheck("pir scan kernel launch");
    if (rc != DPF_AMD_OK) return rc;
  }
  return dpf_amd_xor_fold(workspace, grid, (int64_t)num_queries * record_stride, out, stream);
}

}  // extern "C"
