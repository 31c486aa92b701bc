// aes_device.h — device building blocks shared by the gfx950 kernels: the
// LDS T-table AES core, the DPF PRG steps and the value conversion/correction.
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
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <type_traits>

#include "aes_tables.h"
#include "dpf_amd.h"
#include "internal.h"
#include "kernel_args.h"

#ifndef DPF_AES_SCHED
#define DPF_AES_SCHED 1  // issue a round's table reads as one group
#endif
#ifndef DPF_VALUE_PAIRS
#define DPF_VALUE_PAIRS 1  // AesPairs for the value PRG of even seeds
#endif
#ifndef DPF_BS_LAST
#define DPF_BS_LAST 0  // experiment: the tree pair's last AES round on the VALU
#endif
#if DPF_BS_LAST
#include "bs_last_round.h"
#endif
#ifndef DPF_LANE_WALK
#define DPF_LANE_WALK 1  // divergent walk levels: 1 AES with a per-lane key
#endif

namespace dpf_amd {

// One copy per translation unit (each .hip file is its own code object).
static __constant__ Te0Table c_te0 = MakeTe0();

// ----------------------------------------------------------------------------
// AES core
// ----------------------------------------------------------------------------

struct Lds {
  const char* base;
  uint32_t laneoff;
};

// Table fill.  Row e of the table is 64 words: T0[e] x 32 | T1[e] x 32.
// DPF_FILL_SCALAR (default): wave w of the block writes rows 16w.. in chunks
// of 16, each chunk's 16 entries read by one scalar load (s_load_dwordx16
// through the constant cache, the row index is wave-uniform), then one
// ds_write_b32 per row (lane l -> word l: conflict-free).  The previous
// loop read an entry per word with 64-lane vector loads, eight in flight,
// so a block waited two L2 round trips before its first lookup.
#ifndef DPF_FILL_SCALAR
#define DPF_FILL_SCALAR 1
#endif
template <bool T4>
__device__ __forceinline__ void FillRows(uint32_t* tab) {
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // blockDim.x is a multiple of 64, at most 1024; a block below one wave
  // would otherwise never advance r0
  const int W = max(1, static_cast<int>(blockDim.x >> 6));
  for (int r0 = w * 16; r0 < 256; r0 += W * 16) {
    uint32_t e[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) e[r] = c_te0.t[r0 + r];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const uint32_t v = (lane & 32) ? ((e[r] << 8) | (e[r] >> 24)) : e[r];  // T1 = rotl8(T0)
      tab[(r0 + r) * 64 + lane] = v;
      if (T4) tab[kTabWords + (r0 + r) * 64 + lane] = (v << 16) | (v >> 16);  // T2 / T3
    }
  }
}

__device__ __forceinline__ void FillTables(uint32_t* tab) {
#if DPF_FILL_SCALAR
  FillRows<false>(tab);
#else
  for (int i = threadIdx.x; i < kTabWords; i += blockDim.x) {
    uint32_t v = c_te0.t[i >> 6];
    tab[i] = (i & 32) ? ((v << 8) | (v >> 24)) : v;  // T1 = rotl8(T0)
  }
#endif
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
// post(n, i, w) is applied after round-key word i entered state n's word
// (identity except for per-lane masked keys).
struct KeyNoPost {
  static constexpr bool kBsLast = false;  // keys the VALU last round may use
  __device__ __forceinline__ uint32_t post(int, int, uint32_t w) const { return w; }
};
template <int W>
struct DpfKeyAt : KeyNoPost {  // one fixed DPF key for all states
  // DPF_BS_LAST >= 2: the value PRG pairs' last round on the VALU too
  static constexpr bool kBsLast = DPF_BS_LAST >= 2;
  __device__ __forceinline__ uint32_t rk(int, int i) const { return kDpfKeys[W].rk[i]; }
  __device__ __forceinline__ uint32_t rkr(int, int i) const { return kDpfKeys[W].rkr[i]; }
};
// Key classes that declare kBsLast = true (the tree pair's fixed keys).
template <class K, class = void>
struct BsLastKey : std::false_type {};
template <class K>
struct BsLastKey<K, std::enable_if_t<K::kBsLast>> : std::true_type {};

struct DpfLeftRight : KeyNoPost {  // state 0: left key, state 1: right key
  static constexpr bool kBsLast = true;
  __device__ __forceinline__ uint32_t rk(int n, int i) const { return kDpfKeys[n].rk[i]; }
  __device__ __forceinline__ uint32_t rkr(int n, int i) const { return kDpfKeys[n].rkr[i]; }
};
struct DpfSelect : KeyNoPost {  // wave-uniform choice of the left / right key
  bool right;
  __device__ __forceinline__ uint32_t rk(int, int i) const {
    return right ? kDpfKeys[1].rk[i] : kDpfKeys[0].rk[i];
  }
  __device__ __forceinline__ uint32_t rkr(int, int i) const {
    return right ? kDpfKeys[1].rkr[i] : kDpfKeys[0].rkr[i];
  }
};
struct PairSelect : KeyNoPost {  // generic keys from a kernel argument
  const KeyPair& kp;
  bool right;
  __device__ __forceinline__ uint32_t rk(int, int i) const {
    return right ? kp.k[1].rk[i] : kp.k[0].rk[i];
  }
  __device__ __forceinline__ uint32_t rkr(int, int i) const {
    return right ? kp.k[1].rkr[i] : kp.k[0].rkr[i];
  }
};

// Per-lane choice of the left / right DPF key for N states: every round key
// enters as the left key's word (an SGPR constant) and the lanes taking the
// right key XOR in (left ^ right) under a lane mask — one VALU op per word,
// no per-lane key words held in VGPRs.
struct KeyDiff {
  uint32_t d[44];
};
constexpr KeyDiff MakeKeyDiff() {
  KeyDiff k{};
  for (int i = 0; i < 44; ++i) k.d[i] = kDpfKeys[0].rk[i] ^ kDpfKeys[1].rk[i];
  return k;
}
constexpr KeyDiff kDpfDiff = MakeKeyDiff();
template <int N>
struct DpfMasked {
  uint32_t m[N];  // 0: left key, ~0: right key
  __device__ __forceinline__ uint32_t rk(int, int i) const { return kDpfKeys[0].rk[i]; }
  __device__ __forceinline__ uint32_t rkr(int, int i) const { return kDpfKeys[0].rkr[i]; }
  __device__ __forceinline__ uint32_t post(int n, int i, uint32_t w) const {
    return w ^ (kDpfDiff.d[i] & m[n]);
  }
};

// One full round r (1..9) of one state: the 16 lookups into t, then the
// column combine into w.
__device__ __forceinline__ void RoundLoads(const uint32_t (&w)[4], const Lds& L,
                                           uint32_t (&t)[4][4]) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    t[c][0] = LoadT0(L, w[c], 0);
    t[c][1] = LoadT1(L, w[(c + 1) & 3], 1);
    t[c][2] = LoadT0(L, w[(c + 2) & 3], 2);
    t[c][3] = LoadT1(L, w[(c + 3) & 3], 3);
  }
}
template <class K>
__device__ __forceinline__ void RoundCombine(const uint32_t (&t)[4][4], const K& key, int n,
                                             int r, uint32_t (&w)[4]) {
#pragma unroll
  for (int c = 0; c < 4; ++c)
    w[c] = key.post(n, 4 * r + c,
                    Xor3(t[c][0], t[c][1], Rotl16(Xor3(t[c][2], t[c][3], key.rkr(n, 4 * r + c)))));
}

// N independent AES-128 encryptions in lockstep.  Each round first forms all
// 16N table addresses (v_perm), then issues all 16N ds_read_b32 back to back
// (sched_group_barrier keeps the scheduler from splitting them into small
// waitcnt-separated groups), then combines: per output column
// T0[a] ^ T1[b] ^ rotl16(T0[c] ^ T1[d] ^ rotr16(rk)) = 2 v_bitop3 + 1 alignbit.
// AesFromRound runs rounds R0..10 (the states already hold round R0-1's
// output).
template <int N, int R0, class K>
__device__ __forceinline__ void AesFromRound(uint32_t (&w)[N][4], const K& key,
                                             const Lds& L) {
#pragma unroll
  for (int r = R0; r < 10; ++r) {
    uint32_t t[N][4][4];
#pragma unroll
    for (int n = 0; n < N; ++n) RoundLoads(w[n], L, t[n]);
#if DPF_AES_SCHED
    __builtin_amdgcn_sched_group_barrier(0x002, 16 * N, 0);  // address VALU
    __builtin_amdgcn_sched_group_barrier(0x100, 16 * N, 0);  // DS reads
#endif
#pragma unroll
    for (int n = 0; n < N; ++n) RoundCombine(t[n], key, n, r, w[n]);
  }
#if DPF_BS_LAST
  // (experiment) the tree pair's last round on the VALU:
  // bitsliced SubBytes over both states, then ShiftRows + the round key as
  // two v_perm + one XOR3 per column — no LDS lookups.
  if constexpr (N == 2 && BsLastKey<K>::value) {
    uint32_t R[8] = {w[0][0], w[0][1], w[0][2], w[0][3], w[1][0], w[1][1], w[1][2], w[1][3]};
    BsSubBytes8(R);
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint32_t lo = __builtin_amdgcn_perm(R[4 * n + ((c + 1) & 3)], R[4 * n + c], 0x0c0c0500u);
        const uint32_t hi =
            __builtin_amdgcn_perm(R[4 * n + ((c + 3) & 3)], R[4 * n + ((c + 2) & 3)], 0x07020c0cu);
        w[n][c] = key.post(n, 40 + c, Xor3(lo, hi, key.rk(n, 40 + c)));
      }
    return;
  }
#endif
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
#if DPF_AES_SCHED
  __builtin_amdgcn_sched_group_barrier(0x002, 16 * N, 0);
  __builtin_amdgcn_sched_group_barrier(0x100, 16 * N, 0);
#endif
#pragma unroll
  for (int n = 0; n < N; ++n)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint32_t lo = __builtin_amdgcn_perm(t[n][c][1], t[n][c][0], 0x0c0c0501u);
      const uint32_t hi = __builtin_amdgcn_perm(t[n][c][3], t[n][c][2], 0x07020c0cu);
      w[n][c] = key.post(n, 40 + c, Xor3(lo, hi, key.rk(n, 40 + c)));
    }
}

template <int N, class K>
__device__ __forceinline__ void AesN(uint32_t (&w)[N][4], const K& key,
                                     const Lds& L) {
#pragma unroll
  for (int n = 0; n < N; ++n)
#pragma unroll
    for (int c = 0; c < 4; ++c) w[n][c] = key.post(n, c, w[n][c] ^ key.rk(n, c));
  AesFromRound<N, 1>(w, key, L);
}

// NP pairs of blocks (w[2p], w[2p+1]) where w[2p+1] = w[2p] ^ (1 in bit 0 of
// word 2): the value-PRG inputs sigma(s) and sigma(s + 1) of an even seed s
// (cc:533-537; s + 1 only sets bit 0 of s.lo, i.e. bit 0 of sigma's byte 8).
// After round 1 the odd state differs from the even one in column 2 only
// (one lookup differs: T0 of byte 8); after round 2 each column differs by
// one lookup.  So the odd block costs 1 + 4 lookups for rounds 1-2 instead
// of 32: 133 instead of 160 lookups per odd block.  Keys: one fixed key.
template <int NP, class K>
__device__ __forceinline__ void AesPairs(uint32_t (&w)[2 * NP][4], const K& key,
                                         const Lds& L) {
  uint32_t e[NP][4], t[NP][4][4], x[NP][4];
#pragma unroll
  for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int c = 0; c < 4; ++c) e[p][c] = w[2 * p][c] ^ key.rk(0, c);
  // Round 1: the even block's 16 lookups + T0 of the odd block's byte 8.
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    RoundLoads(e[p], L, t[p]);
    x[p][0] = LoadT0(L, e[p][2] ^ 1u, 0);
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    RoundCombine(t[p], key, 0, 1, e[p]);
#pragma unroll
    for (int c = 0; c < 4; ++c) w[2 * p + 1][c] = e[p][c];
    w[2 * p + 1][2] ^= t[p][2][0] ^ x[p][0];
  }
  // Round 2: the even block's 16 lookups + the 4 lookups of the odd
  // block's column 2, which feeds T0 into column 2, T1 into column 1,
  // T2 = rotl16(T0) into column 0 and T3 = rotl16(T1) into column 3.
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    RoundLoads(e[p], L, t[p]);
    const uint32_t o = w[2 * p + 1][2];
    x[p][0] = LoadT0(L, o, 0);
    x[p][1] = LoadT1(L, o, 1);
    x[p][2] = LoadT0(L, o, 2);
    x[p][3] = LoadT1(L, o, 3);
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    RoundCombine(t[p], key, 0, 2, e[p]);
    w[2 * p + 1][0] = e[p][0] ^ Rotl16(t[p][0][2] ^ x[p][2]);
    w[2 * p + 1][1] = Xor3(e[p][1], t[p][1][1], x[p][1]);
    w[2 * p + 1][2] = Xor3(e[p][2], t[p][2][0], x[p][0]);
    w[2 * p + 1][3] = e[p][3] ^ Rotl16(t[p][3][3] ^ x[p][3]);
#pragma unroll
    for (int c = 0; c < 4; ++c) w[2 * p][c] = e[p][c];
  }
  AesFromRound<2 * NP, 3>(w, key, L);
}

// sigma(x) = (x.hi ^ x.lo, x.hi) (aes_128_fixed_key_hash.cc:75-78) in words.
__device__ __forceinline__ void Sigma(const uint32_t (&x)[4], uint32_t (&s)[4]) {
  s[0] = x[2];
  s[1] = x[3];
  s[2] = x[0] ^ x[2];
  s[3] = x[1] ^ x[3];
}

// ----------------------------------------------------------------------------
// Quad-lane AES: four lanes share one state, lane c holding column c
// (k_walk.hip KEvaluatePointsQuad, expand_device.h KExpandCoop's walk)
// ----------------------------------------------------------------------------

template <int SEL>
__device__ __forceinline__ uint32_t QuadPerm(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, SEL, 0xf, 0xf, false);
}
constexpr int kQuadNext1 = 1 | (2 << 2) | (3 << 4) | (0 << 6);  // lane c <- c+1
constexpr int kQuadNext2 = 2 | (3 << 2) | (0 << 4) | (1 << 6);  // lane c <- c+2
constexpr int kQuadNext3 = 3 | (0 << 2) | (1 << 4) | (2 << 6);  // lane c <- c+3
template <int K>
constexpr int kQuadBcast = K | (K << 2) | (K << 4) | (K << 6);  // lane c <- K

__device__ __forceinline__ uint32_t PickCol(int c, uint32_t a, uint32_t b, uint32_t d,
                                            uint32_t e) {
  return c == 0 ? a : c == 1 ? b : c == 2 ? d : e;
}

// Column c's words of one expanded key: the initial and last round-key word
// and the rotr16 form of rounds 1-9 (the T-table combine's operand).
struct QuadKey {
  uint32_t rk0, rk10, rkr[9];
};
template <int W>
__device__ __forceinline__ QuadKey MakeQuadKey(int c) {
  QuadKey k;
  k.rk0 = PickCol(c, kDpfKeys[W].rk[0], kDpfKeys[W].rk[1], kDpfKeys[W].rk[2], kDpfKeys[W].rk[3]);
  k.rk10 = PickCol(c, kDpfKeys[W].rk[40], kDpfKeys[W].rk[41], kDpfKeys[W].rk[42],
                   kDpfKeys[W].rk[43]);
#pragma unroll
  for (int r = 1; r < 10; ++r)
    k.rkr[r - 1] = PickCol(c, kDpfKeys[W].rkr[4 * r], kDpfKeys[W].rkr[4 * r + 1],
                           kDpfKeys[W].rkr[4 * r + 2], kDpfKeys[W].rkr[4 * r + 3]);
  return k;
}
struct QuadDiff {
  uint32_t d[11];
};
__device__ __forceinline__ QuadDiff MakeQuadDiff(int c) {
  QuadDiff k;
#pragma unroll
  for (int r = 0; r < 11; ++r)
    k.d[r] = PickCol(c, kDpfDiff.d[4 * r], kDpfDiff.d[4 * r + 1], kDpfDiff.d[4 * r + 2],
                     kDpfDiff.d[4 * r + 3]);
  return k;
}

// AES-128 of the quad's state (this lane: column word w); the key of lane
// group = left key, XORed with the left/right difference where m = ~0.
template <bool MASKED>
__device__ __forceinline__ uint32_t AesQuad(uint32_t w, const QuadKey& k, const QuadDiff& d,
                                            uint32_t m, const Lds& L) {
  w ^= k.rk0;
  if (MASKED) w ^= d.d[0] & m;
#pragma unroll
  for (int r = 1; r < 10; ++r) {
    const uint32_t x1 = QuadPerm<kQuadNext1>(w), x2 = QuadPerm<kQuadNext2>(w),
                   x3 = QuadPerm<kQuadNext3>(w);
    const uint32_t t0 = LoadT0(L, w, 0), t1 = LoadT1(L, x1, 1), t2 = LoadT0(L, x2, 2),
                   t3 = LoadT1(L, x3, 3);
    w = Xor3(t0, t1, Rotl16(Xor3(t2, t3, k.rkr[r - 1])));
    if (MASKED) w ^= d.d[r] & m;
  }
  const uint32_t x1 = QuadPerm<kQuadNext1>(w), x2 = QuadPerm<kQuadNext2>(w),
                 x3 = QuadPerm<kQuadNext3>(w);
  const uint32_t t0 = LoadT0(L, w, 0), t1 = LoadT0(L, x1, 1), t2 = LoadT0(L, x2, 2),
                 t3 = LoadT1(L, x3, 3);
  const uint32_t lo = __builtin_amdgcn_perm(t1, t0, 0x0c0c0501u);
  const uint32_t hi = __builtin_amdgcn_perm(t3, t2, 0x07020c0cu);
  w = Xor3(lo, hi, k.rk10);
  if (MASKED) w ^= d.d[10] & m;
  return w;
}

// sigma(x) (aes_128_fixed_key_hash.cc:75-78) by columns: (x2, x3, x0^x2, x1^x3).
__device__ __forceinline__ uint32_t SigmaQuad(uint32_t x, int c) {
  const uint32_t y = QuadPerm<kQuadNext2>(x);
  return c >= 2 ? (x ^ y) : y;
}

// One level of a path walk by a quad (ExpandSeeds / EvaluateSeeds step,
// cc:289-372): child = H_{bit}(sigma(x)) ^ sigma(x) ^ (t ? cw.seed : 0), its
// control bit = LSB ^ (t & cw.control_{bit}), LSB cleared.  cw_word is
// column c of the correction seed.
__device__ __forceinline__ void QuadWalkStep(uint32_t& x, uint32_t& t, uint32_t bit,
                                             uint32_t cw_word, uint32_t cl, uint32_t cr, int c,
                                             const QuadKey& kl, const QuadDiff& kd,
                                             const Lds& L) {
  const uint32_t sg = SigmaQuad(x, c);
  const uint32_t st = AesQuad<true>(sg, kl, kd, 0u - bit, L);
  x = st ^ sg ^ (cw_word & (0u - t));
  const uint32_t lsb = QuadPerm<kQuadBcast<0>>(x) & 1u;
  t = lsb ^ (t & (bit ? cr : cl));
  if (c == 0) x &= ~1u;
}

// ---- latency-bound quad walks (KEvaluatePointsQuad) -------------------------
//
// A quad round is a dependent chain: 3 DPP moves -> 4 v_perm -> 4 ds_read_b32
// -> the combine -> the next round, at one wave per SIMD (one key's 16,384-
// point EvaluateAt).  Two cuts of the chain's post-lookup part:
//  * the per-lane left/right key choice is folded into the round keys once
//    per level (rk ^ (diff & m), off the chain) instead of an XOR after every
//    round (DPF_QUAD_RKM);
//  * four tables instead of two (DPF_QUAD_T4): T2 = rotl16(T0) and T3 =
//    rotl16(T1) stored in a second 64 KiB half (128 KiB per block), so the
//    combine is Xor3(t0, t1, Xor3(t2, t3, rk)) without the rotl16.  The upper
//    half's address comes from the same single v_perm: its lane-offset source
//    carries 0x01 in byte 2 (address bit 16).
#ifndef DPF_QUAD_RKM
#define DPF_QUAD_RKM 1
#endif
#ifndef DPF_QUAD_POSTDPP
#define DPF_QUAD_POSTDPP 2  // 2: moves folded into VOP2 DPP XORs (64 calls 7.38-7.63 -> 7.33-7.39 ms)
#endif
constexpr int kTab4Words = 2 * kTabWords;  // 128 KiB

__device__ __forceinline__ void FillTables4(uint32_t* tab) {
#if DPF_FILL_SCALAR
  FillRows<true>(tab);
#else
  for (int i = threadIdx.x; i < kTab4Words; i += blockDim.x) {
    const int j = i & (kTabWords - 1);
    uint32_t v = c_te0.t[j >> 6];
    if (j & 32) v = (v << 8) | (v >> 24);      // T1 = rotl8(T0)
    if (i >= kTabWords) v = (v << 16) | (v >> 16);  // T2 / T3 = rotl16(T0 / T1)
    tab[i] = v;
  }
#endif
}

struct Lds4 {
  const char* base;
  uint32_t laneoff;     // (lane & 31) * 4
  uint32_t laneoff_hi;  // laneoff | 0x10000: the [T2 | T3] half
};
__device__ __forceinline__ Lds4 MakeLds4(const uint32_t* tab) {
  const uint32_t lo = (threadIdx.x & 31u) * 4u;
  return Lds4{reinterpret_cast<const char*>(tab), lo, lo | 0x10000u};
}
// byte k of x -> address bits 8..15, byte 2 of the lane-offset source -> bits 16..23
#define DPF_SEL_HI(k) (0x0c020000u | ((4u + (k)) << 8))
__device__ __forceinline__ uint32_t LoadT2(const Lds4& L, uint32_t x, int k) {
  const uint32_t a = __builtin_amdgcn_perm(x, L.laneoff_hi, DPF_SEL_HI(k));
  return *reinterpret_cast<const uint32_t*>(L.base + a);
}
__device__ __forceinline__ uint32_t LoadT3(const Lds4& L, uint32_t x, int k) {
  const uint32_t a = __builtin_amdgcn_perm(x, L.laneoff_hi, DPF_SEL_HI(k));
  return *reinterpret_cast<const uint32_t*>(L.base + a + 128);
}

__device__ __forceinline__ Lds LdsOf(const Lds& L) { return L; }
__device__ __forceinline__ Lds LdsOf(const Lds4& L) { return Lds{L.base, L.laneoff}; }

// Column c's plain round-key words of DPF key W (rounds 0..10).
struct QuadRk {
  uint32_t rk[11];
};
template <int W>
__device__ __forceinline__ QuadRk MakeQuadRk(int c) {
  QuadRk k;
#pragma unroll
  for (int r = 0; r < 11; ++r)
    k.rk[r] = PickCol(c, kDpfKeys[W].rk[4 * r], kDpfKeys[W].rk[4 * r + 1],
                      kDpfKeys[W].rk[4 * r + 2], kDpfKeys[W].rk[4 * r + 3]);
  return k;
}
// The level's round keys of this lane: left key, or right where m = ~0.
__device__ __forceinline__ QuadRk MaskQuadRk(const QuadRk& kl, const QuadDiff& d, uint32_t m) {
  QuadRk k;
#pragma unroll
  for (int r = 0; r < 11; ++r) k.rk[r] = kl.rk[r] ^ (d.d[r] & m);
  return k;
}

// AES-128 of the quad's state with per-lane round keys `k` (plain words).
// T4: four tables (Lds4); otherwise T0/T1 with the rotl16 in the combine.
template <bool T4, class LT>
__device__ __forceinline__ uint32_t AesQuadRk(uint32_t w, const QuadRk& k, const LT& L) {
  w ^= k.rk[0];
#pragma unroll
  for (int r = 1; r < 10; ++r) {
    if constexpr (T4 && DPF_QUAD_POSTDPP) {
      // lookups on this lane's own bytes first, the moves after: lane c's
      // T_k[byte k of column c] is what lane c - k needs.  The chain of a
      // round is v_perm -> ds_read -> (3 DPP-sourced ops) -> xor3, one VALU
      // level shorter than moving the column words before the lookups (and no
      // VALU-write -> DPP-read wait states on w).
      const uint32_t u0 = LoadT0(LdsOf(L), w, 0), u1 = LoadT1(LdsOf(L), w, 1),
                     u2 = LoadT2(L, w, 2), u3 = LoadT3(L, w, 3);
#if DPF_QUAD_POSTDPP >= 2
      // the moves folded into the XORs' first operand (VOP2 DPP); u1 / u3
      // come from ds_read, so no VALU-write -> DPP-read wait state applies
      uint32_t a, b;
      asm("v_xor_b32_dpp %0, %1, %2 quad_perm:[1,2,3,0] row_mask:0xf bank_mask:0xf"
          : "=v"(a) : "v"(u1), "v"(u0));
      asm("v_xor_b32_dpp %0, %1, %2 quad_perm:[3,0,1,2] row_mask:0xf bank_mask:0xf"
          : "=v"(b) : "v"(u3), "v"(k.rk[r]));
#else
      const uint32_t a = QuadPerm<kQuadNext1>(u1) ^ u0;
      const uint32_t b = QuadPerm<kQuadNext3>(u3) ^ k.rk[r];
#endif
      w = Xor3(a, b, QuadPerm<kQuadNext2>(u2));
      continue;
    }
    const uint32_t x1 = QuadPerm<kQuadNext1>(w), x2 = QuadPerm<kQuadNext2>(w),
                   x3 = QuadPerm<kQuadNext3>(w);
    if constexpr (T4) {
      const uint32_t t0 = LoadT0(LdsOf(L), w, 0),
                     t1 = LoadT1(LdsOf(L), x1, 1), t2 = LoadT2(L, x2, 2),
                     t3 = LoadT3(L, x3, 3);
      w = Xor3(t0, t1, Xor3(t2, t3, k.rk[r]));
    } else {
      const uint32_t t0 = LoadT0(L, w, 0), t1 = LoadT1(L, x1, 1), t2 = LoadT0(L, x2, 2),
                     t3 = LoadT1(L, x3, 3);
      // rotl16(t2 ^ t3 ^ rotr16(rk)) = rotl16(t2 ^ t3) ^ rk
      w = Xor3(t0, t1, Rotl16(Xor3(t2, t3, __builtin_amdgcn_alignbit(k.rk[r], k.rk[r], 16))));
    }
  }
  const Lds L2 = LdsOf(L);
  const uint32_t x1 = QuadPerm<kQuadNext1>(w), x2 = QuadPerm<kQuadNext2>(w),
                 x3 = QuadPerm<kQuadNext3>(w);
  const uint32_t t0 = LoadT0(L2, w, 0), t1 = LoadT0(L2, x1, 1), t2 = LoadT0(L2, x2, 2),
                 t3 = LoadT1(L2, x3, 3);
  const uint32_t lo = __builtin_amdgcn_perm(t1, t0, 0x0c0c0501u);
  const uint32_t hi = __builtin_amdgcn_perm(t3, t2, 0x07020c0cu);
  return Xor3(lo, hi, k.rk[10]);
}

// QuadWalkStep with the level's keys folded once (rk ^ (diff & m)).
template <bool T4, class LT>
__device__ __forceinline__ void QuadWalkStepRk(uint32_t& x, uint32_t& t, uint32_t bit,
                                               uint32_t cw_word, uint32_t cl, uint32_t cr, int c,
                                               const QuadRk& kl, const QuadDiff& kd,
                                               const LT& L) {
  const QuadRk k = MaskQuadRk(kl, kd, 0u - bit);
  const uint32_t sg = SigmaQuad(x, c);
  const uint32_t st = AesQuadRk<T4>(sg, k, L);
  x = st ^ sg ^ (cw_word & (0u - t));
  const uint32_t lsb = QuadPerm<kQuadBcast<0>>(x) & 1u;
  t = lsb ^ (t & (bit ? cr : cl));
  if (c == 0) x &= ~1u;
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

struct ExpandCtx {
  const ExpandArgs& a;
  const VtDev& vt;
  const Lds& L;
  // batched keys: this block's key's packed value correction and party
  // (EmitDirect); otherwise vt.corr_packed / vt.party apply
  bool per_key = false;
  uint32_t kcorr[4] = {0u, 0u, 0u, 0u};
  int kparty = 0;
  int64_t cw0 = 0;  // first correction word of this key ([key][level] layout)
};

// Value PRG of one seed: block j = H_value(seed + j) (cc:523-547).
// kEven: every seed has bit 0 clear (a seed whose control bit was just
// extracted), so blocks (2i, 2i+1) go through AesPairs.
template <int NS, int BN, bool kEven = false>
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
  if constexpr (kEven && BN % 2 == 0 && DPF_VALUE_PAIRS) {
    AesPairs<NS * BN / 2>(st, DpfKeyAt<2>{}, L);
  } else {
    AesN<NS * BN>(st, DpfKeyAt<2>{}, L);
  }
#pragma unroll
  for (int n = 0; n < NS; ++n)
#pragma unroll
    for (int j = 0; j < BN; ++j)
#pragma unroll
      for (int c = 0; c < 4; ++c) h[n][j][c] = st[n * BN + j][c] ^ sg[n * BN + j][c];
}

}  // namespace dpf_amd
