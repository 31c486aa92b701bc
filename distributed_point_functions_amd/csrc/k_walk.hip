// k_walk.hip — path-walk kernels: EvaluateSeeds (evaluate_prg_hwy.cc:552-634),
// the fused EvaluateAt / EvaluateAndApply point evaluation and the plain
// AES-MMO hash (aes_128_fixed_key_hash.cc:57-98).
#include "aes_device.h"

namespace dpf_amd {

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

int LaunchEvaluateSeeds(int grid, hipStream_t st, const WalkArgs& a, const KeyPair& kp) {
  hipLaunchKernelGGL(KEvaluateSeeds, dim3(grid), dim3(kBlock), 0, st, a, kp);
  return LaunchCheck("evaluate_seeds kernel launch");
}

int LaunchEvaluatePoints(int bn, int grid, hipStream_t st, const PointsArgs& a,
                         const VtDev& vt) {
  switch (bn) {
    case 1:
      hipLaunchKernelGGL((KEvaluatePoints<1>), dim3(grid), dim3(kBlock), 0, st, a, vt);
      break;
    case 2:
      hipLaunchKernelGGL((KEvaluatePoints<2>), dim3(grid), dim3(kBlock), 0, st, a, vt);
      break;
    default:
      hipLaunchKernelGGL((KEvaluatePoints<4>), dim3(grid), dim3(kBlock), 0, st, a, vt);
  }
  return LaunchCheck("evaluate_points kernel launch");
}

int LaunchAesMmo(int grid, hipStream_t st, const uint4* in, uint4* out, int64_t n,
                 const KeyPair& kp) {
  hipLaunchKernelGGL(KAesMmo, dim3(grid), dim3(kBlock), 0, st, in, out, n, kp);
  return LaunchCheck("aes kernel launch");
}

}  // namespace dpf_amd
