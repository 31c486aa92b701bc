// kernels_capi.cc — the Tier-1 C ABI (include/dpf_amd.h): argument checks
// with the reference's messages, device descriptors, grid sizing, and the
// calls into the kernel launchers of k_*.hip.  No device code lives here.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "aes_tables.h"
#include "dpf_amd.h"
#include "internal.h"
#include "kernel_args.h"
#include "host_device.h"

// D = 3 for the KExpand depth A/B (tools/ab_c3_depth.sh); the product build
// instantiates D in {0, 1, 2, 4, 5, 6, 8}.
#ifndef DPF_EXPAND_EXTRA_DEPTHS
#define DPF_EXPAND_EXTRA_DEPTHS 0
#endif

namespace dpf_amd {

namespace {

// Test hooks, per calling thread: a test forcing a kernel variant never
// changes what another thread's launches pick.
thread_local int t_expand_depth = 0;  // dpf_amd_set_expand_depth
thread_local int t_walk_mode = 0;     // dpf_amd_set_walk_mode
// dpf_amd_set_expand_roots: -1 automatic, 0 off, 1 whenever eligible.
// DPF_AMD_EXPAND_ROOTS=0 starts every thread with it off (A/B runs).
const int kExpandRootsDefault = [] {
  const char* e = std::getenv("DPF_AMD_EXPAND_ROOTS");
  return (e && std::atoi(e) == 0) ? 0 : -1;
}();
thread_local int t_expand_roots = kExpandRootsDefault;
thread_local int t_dcf_generic = 0;   // dpf_amd_set_dcf_kernel
// dpf_amd_set_scan_m4; the process default comes from DPF_AMD_SCAN_M4 (A/B runs)
const int kScanM4Default = [] {
  const char* e = std::getenv("DPF_AMD_SCAN_M4");
  return e ? std::atoi(e) : -1;
}();
thread_local int t_scan_m4 = kScanM4Default;
// dpf_amd_set_scan_skip_unselected (opt-in): the masked scan reads only the
// records some query of the pass selects, as the reference's scan does
// (inner_product_hwy.cc:213-221).  Off by default: every record is read, so
// the scan's access pattern does not depend on the selection share.
const int kScanSkipDefault = [] {
  const char* e = std::getenv("DPF_AMD_SCAN_SKIP_UNSELECTED");
  return (e && std::atoi(e) != 0) ? 1 : 0;
}();
thread_local int t_scan_skip = kScanSkipDefault;

int GridFor(int64_t items, int block, int max_blocks) {
  int64_t g = (items + block - 1) / block;
  if (g < 1) g = 1;
  if (g > max_blocks) g = max_blocks;
  return (int)g;
}

// Kernel for a single-key launch of `leaves` tree leaves of a tree of >= 11
// levels, from tools/expand_sweep.py on MI355X (profiles/sweep_*_r03i.log,
// KExpandCoop with its quad-lane walk to the block root): below 2^22 leaves
// the launch is latency-bound (one block of 2^11 leaves takes 22 us with the
// launch) and KExpandCoop computes each tree node once — 2^19 leaves (c1, a
// PIR selection): 38 us against KExpand<2> 59 and KExpand<4> 111; 2^21:
// E = 1 0.108 ms against KExpand<4> 0.125; from 2^23 KExpand<4>'s
// full-occupancy register DFS wins (0.358 vs 0.384 ms) until KExpand<8> at
// 2^25.
// Round 5 (tools/expand_sweep.py, profiles/sweep_single_r05v.log): up to
// 2^16 leaves 256-leaf blocks (E = -2: the 1024 and 512-node levels and the
// one-lane hashes replaced by the value hash on quads) — 2^11 13.4 vs 18.2 us,
// 2^16 17.4 vs 21.7 us (the c4/8 PIR selection); level at 2^17, behind above.
int CoopDepth(int64_t leaves) {
  return leaves >= (int64_t{1} << 19) ? -2 : leaves > (int64_t{1} << 16) ? -1 : -3;
}
// log2 leaves per thread (KExpand, D >= 0) or per block: D = -1 / -2 / -3 are
// KExpandCoop with E = 0 / 1 / -2 (1024 / 2048 / 256 leaves per block).
int CoopSub(int D) { return D >= 0 ? D : D == -3 ? 8 : 9 - D; }
constexpr int64_t kCoopMaxLeaves = int64_t{1} << 22;

// Kernel for a batched expansion of num_keys x range tree leaves
// (tools/expand_sweep.py batched, profiles/sweep_batched_r03m.log): from 2^23
// leaves in total KExpand<6> with per-lane keys for 16-byte elements (the
// PIR selection: 64 keys x 2^19 1.09 ms = 0.75 of the LDS
// bound against KExpand<4> 1.32 and the cooperative 1.42; 16 x 2^19 0.377
// vs 0.392), else KExpand<4>; KExpandCoop with per-block keys below (8 x
// 2^19: 0.212 vs D = 4 0.224, D = 6 0.379; 100 x 2^16: 0.316 vs 0.368).
// Depth of a batched expansion: the deepest DFS that still fills one round
// of resident blocks (2^18 threads) — D = 6 from 2^24 leaves in total for
// the 16-byte selection type, D = 5 from 2^23 — else D = 4 or the
// cooperative kernel.  With the wave priority on, 16 keys x 2^19 leaves
// (2^23): D = 4 / 5 / 6 0.360 / 0.305 / 0.347 ms; 64 x 2^19: 1.267 / 1.080 /
// 1.032 ms (profiles/sweep_batched_r06.log).
int BatchedDepth(int64_t num_keys, int64_t range, bool wide) {
  const int64_t total = num_keys * range;
  if (total >= (int64_t{1} << 24) && range >= 64 && wide) return 6;
  if (total >= (int64_t{1} << 23) && range >= 32) return 5;
  if (total >= (int64_t{1} << 23) && range >= 16) return 4;
  return CoopDepth(total);
}

bool SingleDirect(const VtDev& vt) {
  return vt.direct && vt.ns == 1 && vt.sc[0].in_off == 0 && vt.sc[0].out_off == 0 &&
         vt.stride == vt.sc[0].bytes && vt.bn == 1 && vt.epb * vt.sc[0].bytes == 16;
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

// Picks the emitter for the value type.
int LaunchExpandForType(int D, int grid, hipStream_t st, const ExpandArgs& a,
                        const VtDev& vt) {
  if (SingleDirect(vt)) {
    switch (vt.sc[0].bytes) {
      case 1:
        return LaunchExpandDirect1(D, grid, st, a, vt);
      case 2:
        return LaunchExpandDirect2(D, grid, st, a, vt);
      case 4:
        return LaunchExpandDirect4(D, grid, st, a, vt);
      case 8:
        return LaunchExpandDirect8(D, grid, st, a, vt);
      default:
        return LaunchExpandDirect16(D, grid, st, a, vt);
    }
  }
  const bool u32_modn64 =
      !vt.direct && vt.ns == 2 && vt.bn == 2 && vt.epb == 1 &&
      vt.sc[0].kind == DPF_AMD_KIND_INTEGER && vt.sc[0].bytes == 4 &&
      vt.sc[1].kind == DPF_AMD_KIND_INT_MOD_N && vt.sc[1].bytes == 8 &&
      vt.sc[1].use_fold && vt.sc[1].fold_w == 64 && (vt.sc[1].fold_c >> 56) == 0;
  if (u32_modn64) return LaunchExpandU32ModN64(D, grid, st, a, vt);
  switch (BnTemplate(vt.bn)) {
    case 1:
      return LaunchExpandGeneric1(D, grid, st, a, vt);
    case 2:
      return LaunchExpandGeneric2(D, grid, st, a, vt);
    default:
      return LaunchExpandGeneric4(D, grid, st, a, vt);
  }
}

}  // namespace

int WalkMode() { return t_walk_mode; }
bool DcfDirectEnabled() { return t_dcf_generic == 0; }

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

// DPF_AMD_SOURCE_HASH: SHA-256 of the sources and build flags this library
// was compiled from (build_native.source_hash()); build() recompiles when it
// differs from the tree's, and bench.py reports both.
#ifndef DPF_AMD_SOURCE_HASH
#define DPF_AMD_SOURCE_HASH "unknown"
#endif
const char* dpf_amd_version(void) {
  return "dpf_amd 0.1 (gfx950, T-table AES in LDS) src:" DPF_AMD_SOURCE_HASH;
}

int dpf_amd_device_count(int* count) {
  return HipCheck(hipGetDeviceCount(count), "hipGetDeviceCount");
}

int dpf_amd_aes128_mmo(uint64_t key_lo, uint64_t key_hi, const void* in, void* out,
                       int64_t n, void* stream) {
  if (n < 0) return SetError(DPF_AMD_INVALID_ARGUMENT, "negative size");
  if (n == 0) return DPF_AMD_OK;
  if (!in || !out) return SetError(DPF_AMD_INVALID_ARGUMENT, "null buffer");
  KeyPair kp = MakeKeyPair(key_lo, key_hi, key_lo, key_hi);
  return LaunchAesMmo(GridFor(n, kBlock, 2048), (hipStream_t)stream, (const uint4*)in,
                      (uint4*)out, n, kp);
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
  WalkArgs a{};
  a.path_offset = 0;
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
  a.points_per_key = 0;
  a.num_levels = num_levels;
  a.rightshift = paths_rightshift;
  KeyPair kp = MakeKeyPair(key_left_lo, key_left_hi, key_right_lo, key_right_hi);
  if (key_left_lo == kPrgKeyLeftLo && key_left_hi == kPrgKeyLeftHi &&
      key_right_lo == kPrgKeyRightLo && key_right_hi == kPrgKeyRightHi)
    return LaunchEvaluateSeedsDpf(num_seeds, (hipStream_t)stream, a, kp);
  return LaunchEvaluateSeeds(num_seeds, (hipStream_t)stream, a, kp);
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
  // For small problems prefer more threads over deep DFS.  A D = 8 thread
  // expands 256 leaves in sequence (~1.3 ms however small the launch), so
  // D = 8 needs 2^17 threads to beat D = 4 (tools/c1_depth_sweep.py, uint64:
  // 2^24 tree leaves D = 8 1.32 ms vs D = 4 0.80; 2^25: 1.33 vs 1.46), and
  // D = 4 needs 2^16 (2^19 tree leaves: D = 2 0.059 ms vs D = 4 0.112).
  const int64_t range = leaf_end - leaf_begin;
  // With the wave priority, the deepest DFS whose threads still fill one
  // round of resident blocks (2^18 threads) wins: D = 8 from 2^26 tree
  // leaves, D = 6 from 2^24 (uint64, 2^25 leaves: D = 4 / 5 / 6 / 8 1.33 /
  // 1.11 / 1.03 / 1.26 ms; 2^24: 0.77 / 0.59 / 0.53 / 1.24; 2^26: D = 6 2.07,
  // D = 8 2.00; profiles/sweep_large_r06.log).
  if (D == 8 && (range >> 8) < (int64_t{1} << 18))
    D = (range >> 6) >= (int64_t{1} << 18) ? 6 : 4;
  if (D == 4 && (range >> 4) < (int64_t{1} << 16)) D = 2;
  // From 2^18 threads at D = 5 (one full round of resident blocks) the
  // shallower walk beats D = 4's two rounds: c3's 2^16 prefix roots x 7
  // levels 0.290-0.292 -> 0.271-0.274 ms, 2^17 roots 0.519-0.527 ->
  // 0.480-0.483 ms; 2^15 roots (half a round) stay at D = 4 (0.160 against
  // 0.177; profiles/ab_c3_depth5_r06/, with the wave priority).
  if (D == 4 && num_levels >= 5 && (range >> 5) >= (int64_t{1} << 18)) D = 5;
  // Below 2^25 tree leaves the cooperative kernel computes every tree node
  // once per block instead of one root walk per thread (KExpandCoop,
  // expand_device.h): D = -1 (1024 leaves per block) or -2 (2048).
  if (num_levels >= 11 && range < kCoopMaxLeaves) D = CoopDepth(range);
  const int forced = t_expand_depth;
  if (forced > 0 && forced <= num_levels) D = forced;
  if (forced < 0 && num_levels >= CoopSub(forced)) D = forced;
  if (D > num_levels) D = num_levels >= 4 ? 4 : num_levels;
  ExpandArgs a{};
  a.root_seeds = (const uint4*)root_seeds;
  a.root_cb = root_control_bits;
  a.cw_seed = (const uint4*)correction_seeds;
  a.ccl = ccl;
  a.ccr = ccr;
  a.out = (char*)out;
  const int sub = CoopSub(D);  // log2 leaves per thread (KExpand) or per block (coop)
  a.walk = num_levels - sub;
  a.root_level = 0;
  a.root_base = 0;
  a.chunk_begin = leaf_begin >> sub;
  a.chunk_end = (leaf_end + (1ll << sub) - 1) >> sub;
  a.leaf_begin = leaf_begin;
  a.leaf_end = leaf_end;
  a.num_levels = num_levels;
  a.num_keys = 1;
  // Precomputed subtree roots (D = 8 launches of >= 2^28 leaves, c5): every
  // KExpand thread used to walk `walk` levels from the key's root to its
  // subtree root, one AES per level — 24 levels per 256 leaves at c5, 15 of
  // its 615 T-table lookups per leaf.  The levels above the last six are
  // instead computed once per node, by KExpandCoop<0, EmitNodes> (every node
  // of level R = walk - 6 of the launch's range, breadth-first in LDS), and
  // each thread walks only the six levels its wave's lanes differ in.
  hipStream_t st = (hipStream_t)stream;
  constexpr int kCoopLog0 = 10;  // KExpandCoop<0>: 1024 nodes per block
  distributed_point_functions::dpf_internal_host::DeviceBuffer roots;
  const int roots_mode = t_expand_roots;
  if (D == 8 && (forced == 0 || forced == 8) && roots_mode != 0 && a.walk >= 6 + 11 &&
      (roots_mode > 0 || range >= (int64_t{1} << 28))) {
    const int R = a.walk - 6;
    const int64_t rb = a.chunk_begin >> 6, re = ((a.chunk_end - 1) >> 6) + 1;
    distributed_point_functions::Status ast = roots.Alloc(size_t(16) * (re - rb), st);
    if (!ast.ok()) return SetError(ast.raw_code(), ast.message());
    ExpandArgs r{};
    r.root_seeds = a.root_seeds;
    r.root_cb = a.root_cb;
    r.cw_seed = a.cw_seed;
    r.ccl = a.ccl;
    r.ccr = a.ccr;
    r.out = roots.as<char>();
    r.walk = R - kCoopLog0;
    r.chunk_begin = rb >> kCoopLog0;
    r.chunk_end = (re + (int64_t{1} << kCoopLog0) - 1) >> kCoopLog0;
    r.leaf_begin = rb;
    r.leaf_end = re;
    r.num_levels = R;
    r.num_keys = 1;
    rc = LaunchExpandNodes(st, r, dev);
    if (rc != DPF_AMD_OK) return rc;
    a.root_seeds = roots.as<const uint4>();
    a.root_cb = nullptr;
    a.root_base = rb;
    a.root_level = R;
    a.walk = 6;
  }
  // LaunchExpand caps the grid (DPF_EXPAND_MAX_GRID).
  const int grid = GridFor(a.chunk_end - a.chunk_begin, kExpandBlock, INT32_MAX);
  return LaunchExpandForType(D, grid, st, a, dev);
}

int dpf_amd_expand_and_correct_batched(int64_t num_keys, const void* root_seeds,
                                       const uint8_t* root_control_bits, int num_levels,
                                       const void* correction_seeds, const uint8_t* ccl,
                                       const uint8_t* ccr, const dpf_amd_value_type* vt,
                                       const uint64_t* value_corrections, const int8_t* parties,
                                       int corrected_elements_per_block, int64_t leaf_begin,
                                       int64_t leaf_end, void* out, void* stream) {
  if (num_keys < 0 || !vt || num_levels < 0 || num_levels > 62)
    return SetError(DPF_AMD_INVALID_ARGUMENT, "bad arguments");
  if (leaf_begin < 0 || leaf_end > (int64_t{1} << num_levels) || leaf_begin > leaf_end)
    return SetError(DPF_AMD_INVALID_ARGUMENT, "leaf range out of bounds");
  if (num_keys == 0 || leaf_begin == leaf_end) return DPF_AMD_OK;
  const int per = vt->elements_per_block * vt->num_scalars;  // correction words per key
  VtDev probe;
  int rc = MakeVtDev(*vt, nullptr, 0, corrected_elements_per_block, &probe);
  if (rc != DPF_AMD_OK) return rc;
  const int64_t range = leaf_end - leaf_begin;
  hipStream_t st = (hipStream_t)stream;
  if (!SingleDirect(probe) || num_levels < 11 || range >= (int64_t{1} << 25)) {
    // one launch per key (a type whose correction is not one packed block,
    // or keys large enough to fill the GPU on their own)
    const int64_t out_bytes = range * corrected_elements_per_block * vt->out_stride;
    for (int64_t k = 0; k < num_keys; ++k) {
      rc = dpf_amd_expand_and_correct(
          1, static_cast<const char*>(root_seeds) + 16 * k, root_control_bits + k, num_levels,
          static_cast<const char*>(correction_seeds) + 16 * k * num_levels, ccl + k * num_levels,
          ccr + k * num_levels, vt, value_corrections + 2 * per * k, parties[k],
          corrected_elements_per_block, leaf_begin, leaf_end,
          static_cast<char*>(out) + k * out_bytes, stream);
      if (rc != DPF_AMD_OK) return rc;
    }
    return DPF_AMD_OK;
  }
  std::vector<uint64_t> host(2 * num_keys + (num_keys + 15) / 16 * 2, 0);
  for (int64_t k = 0; k < num_keys; ++k) {
    rc = PackedCorrection(*vt, value_corrections + 2 * per * k, corrected_elements_per_block,
                          &host[2 * k]);
    if (rc != DPF_AMD_OK) return rc;
  }
  memcpy(&host[2 * num_keys], parties, num_keys);
  namespace h = distributed_point_functions::dpf_internal_host;
  h::DeviceBuffer dev;
  distributed_point_functions::Status ust = dev.Upload(host.data(), 8 * host.size(), st);
  if (!ust.ok()) return SetError(ust.raw_code(), ust.message());
  return ExpandBatched(num_keys, root_seeds, root_control_bits, num_levels, correction_seeds, ccl,
                       ccr, vt, dev.get(),
                       reinterpret_cast<const int8_t*>(dev.as<char>() + 16 * num_keys),
                       corrected_elements_per_block, leaf_begin, leaf_end, out, stream);
}

int dpf_amd_set_expand_depth(int depth) {
  const bool extra = DPF_EXPAND_EXTRA_DEPTHS && depth == 3;
  if (depth != 0 && depth != 1 && depth != 2 && depth != 4 && depth != 5 && depth != 6 &&
      depth != 8 && depth != -1 && depth != -2 && depth != -3 && !extra)
    return -99;
  const int old = t_expand_depth;
  t_expand_depth = depth;
  return old;
}

int dpf_amd_set_expand_roots(int mode) {
  if (mode < -1 || mode > 1) return -2;
  const int old = t_expand_roots;
  t_expand_roots = mode;
  return old;
}

int dpf_amd_set_dcf_kernel(int mode) {
  if (mode < 0 || mode > 1) return -2;
  const int old = t_dcf_generic;
  t_dcf_generic = mode;
  return old;
}

int dpf_amd_set_walk_mode(int mode) {
  if (mode < 0 || mode > 2) return -2;
  const int old = t_walk_mode;
  t_walk_mode = mode;
  return old;
}

int dpf_amd_set_scan_skip_unselected(int on) {
  if (on != 0 && on != 1) return -2;
  const int old = t_scan_skip;
  t_scan_skip = on;
  return old;
}

int dpf_amd_set_scan_m4(int mode) {
  if (mode < -1 || mode > 1) return -2;
  const int old = t_scan_m4;
  t_scan_m4 = mode;
  return old;
}

// Shared body of dpf_amd_evaluate_points{,_batched}.
static int EvaluatePoints(int64_t num_points, int64_t points_per_key, int64_t num_cw,
                          const void* seeds, const uint8_t* control_bits, const void* paths,
                          int paths_rightshift, int num_levels, const void* correction_seeds,
                          const uint8_t* ccl, const uint8_t* ccr, const dpf_amd_value_type* vt,
                          const uint8_t* block_index, const int8_t* party, int party_all,
                          const void* value_corrections, const uint64_t* value_correction_all,
                          void* out, void* seeds_out, uint8_t* control_bits_out,
                          void* stream, int64_t path_offset = 0,
                          const int32_t* key_index = nullptr, bool seeds_by_key = false) {
  if (num_points < 0 || num_levels < 0 || !vt)
    return SetError(DPF_AMD_INVALID_ARGUMENT, "bad arguments");
  if (num_points == 0) return DPF_AMD_OK;
  VtDev dev;
  int rc = MakeVtDev(*vt, value_correction_all, party_all, vt->elements_per_block, &dev);
  if (rc != DPF_AMD_OK) return rc;
  PointsArgs a{};
  a.w.num_seeds = num_points;
  a.w.num_cw = num_cw;
  a.w.seeds_in = (const uint4*)seeds;
  a.w.cb_in = control_bits;
  a.w.paths = (const uint4*)paths;
  a.w.cw_seed = (const uint4*)correction_seeds;
  a.w.ccl = ccl;
  a.w.ccr = ccr;
  a.w.seeds_out = (uint4*)seeds_out;
  a.w.cb_out = control_bits_out;
  a.w.points_per_key = points_per_key;
  a.w.num_levels = num_levels;
  a.w.rightshift = paths_rightshift;
  a.w.path_offset = path_offset;
  a.w.key_index = key_index;
  a.w.seeds_by_key = seeds_by_key ? 1 : 0;
  a.block_index = block_index;
  a.party = party;
  a.value_corrections = (const uint4*)value_corrections;
  a.out = (char*)out;
  return LaunchEvaluatePoints(BnTemplate(dev.bn), num_points, (hipStream_t)stream, a, dev);
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
  return EvaluatePoints(num_seeds, 0, num_correction_words, seeds, control_bits, paths,
                        paths_rightshift, num_levels, correction_seeds, ccl, ccr, vt,
                        block_index, party, party_all, value_corrections, value_correction_all,
                        out, seeds_out, control_bits_out, stream);
}

int dpf_amd_evaluate_points_batched(int64_t num_keys, int64_t points_per_key,
                                    const void* key_seeds, const uint8_t* key_control_bits,
                                    const void* paths, int paths_rightshift, int num_levels,
                                    const void* correction_seeds, const uint8_t* ccl,
                                    const uint8_t* ccr, const dpf_amd_value_type* vt,
                                    const uint8_t* block_index, const int8_t* key_party,
                                    int party_all, const void* key_value_corrections,
                                    const uint64_t* value_correction_all, void* out,
                                    void* stream) {
  if (num_keys < 0 || points_per_key < 0)
    return SetError(DPF_AMD_INVALID_ARGUMENT, "`num_keys` and `points_per_key` must be >= 0");
  if (num_keys > 0 && points_per_key > INT64_MAX / num_keys)
    return SetError(DPF_AMD_INVALID_ARGUMENT, "too many points");
  if (num_keys == 0 || points_per_key == 0) return DPF_AMD_OK;
  return EvaluatePoints(num_keys * points_per_key, points_per_key, num_keys * num_levels,
                        key_seeds, key_control_bits, paths, paths_rightshift, num_levels,
                        correction_seeds, ccl, ccr, vt, block_index, key_party, party_all,
                        key_value_corrections, value_correction_all, out, nullptr, nullptr,
                        stream);
}

}  // extern "C"

#ifndef DPF_SCAN_GRID_WIDE
#define DPF_SCAN_GRID_WIDE 1
#endif
static int ScanGrid(int64_t num_records, int num_queries, int64_t record_stride) {
  // At least one 128-record tile per wave; up to 8192 blocks / partials
  // (c4 Q = 8: 2.95 ms vs 3.17 ms at 2048 — more, shorter blocks balance
  // across CUs; KPirScanM4 at Q = 100: 2621 waves for 2048 resident slots
  // left a 28 % second round), but at most 256 MiB of partials (grid x
  // queries x record bytes) for the fold, and never fewer than 2048.
  const int64_t tiles = (num_records + 127) / 128;
  const int64_t g = (tiles + kScanWaves - 1) / kScanWaves;
  const int64_t per_block = std::max<int64_t>(1, (int64_t)num_queries * record_stride);
  // Rows wider than one masked-scan slice (64 chunks) multiply the blocks by
  // their slices, so the floor that keeps the CUs busy divides by them
  // (DPF_SCAN_GRID_WIDE): 16 KiB rows at Q = 100 write 0.4 GB of partials
  // instead of 3.4 GB (the fold reads 0.8 GB instead of 6.7).
  const int64_t slices = DPF_SCAN_GRID_WIDE ? std::max<int64_t>(1, (record_stride / 16 + 63) / 64) : 1;
  const int64_t floor = std::max<int64_t>(256, 2048 / slices);
  const int64_t cap = std::max<int64_t>(floor, std::min<int64_t>(8192, (256ll << 20) / per_block));
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}

// Whether the next pass over `rem` queries of C-chunk records runs the
// Four-Russians scan (KPirScanM4*) rather than the masked scan (KPirScanG).
// Mode (dpf_amd_set_scan_m4 / DPF_AMD_SCAN_M4): 0 never, 1 always (tests),
// -1 from kScanM4MinQueries queries on.
static bool UseScanM4(int rem, int C) {
  const int mode = t_scan_m4;
  if (mode == 0) return false;
  if (C > (1 << 16)) return false;  // records > 1 MiB: 128-record tiles past 2^27 B
  if (mode < 0 && (rem < kScanM4MinQueries || C < 4)) return false;
  return true;
}

namespace dpf_amd {
// DPF_AMD_SCAN_SLOTS=0 (A/B): the masked scan always writes one partial per
// block.
static const bool kScanSlotsOn = [] {
  const char* e = std::getenv("DPF_AMD_SCAN_SLOTS");
  return !(e && std::atoi(e) == 0);
}();

ScanPlan PlanScan(int64_t num_records, int64_t record_stride, int num_queries) {
  ScanPlan p;
  p.grid = ScanGrid(num_records, num_queries, record_stride);
  const int C = record_stride > 0 ? (int)(record_stride / 16) : 1;
  // slots only when every pass is a masked pass (KPirScanM4 writes one
  // partial per wave) and the block's partial is small
  p.slots = kScanSlotsOn && num_queries > 0 && !UseScanM4(num_queries, C) &&
            (int64_t)num_queries * record_stride <= kScanSlotMaxBytes && p.grid >= kScanSlots;
  return p;
}

int ScanFoldParts(const ScanPlan& plan) { return plan.slots ? kScanSlots : plan.grid; }

int XorFoldClear(void* parts, int num_parts, int64_t bytes, void* out, void* stream) {
  if (num_parts <= 0 || bytes <= 0) return DPF_AMD_OK;
  hipStream_t st = (hipStream_t)stream;
  if (bytes % 16 == 0 && ((uintptr_t)parts % 16 == 0) && ((uintptr_t)out % 16 == 0)) {
    const int64_t words = bytes / 16;
    const int64_t blocks = (words + kFoldWords - 1) / kFoldWords;
    if (blocks > INT32_MAX) return SetError(DPF_AMD_INVALID_ARGUMENT, "xor fold too large");
    return LaunchXorFold((unsigned)blocks, st, (const uint4*)parts, num_parts, words,
                         (uint4*)out, (uint4*)parts);
  }
  const int rc = dpf_amd_xor_fold(parts, num_parts, bytes, out, stream);
  if (rc != DPF_AMD_OK) return rc;
  return HipCheck(hipMemsetAsync(parts, 0, (size_t)num_parts * bytes, st), "fold slots clear");
}

int ScanPiece(const void* db, int64_t num_records, int64_t record_stride,
              const void* selections, int64_t selection_blocks, int num_queries,
              const ScanPlan& plan, void* partials, void* stream) {
  hipStream_t st = (hipStream_t)stream;
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
  const int C = (int)(record_stride / 16);
  const int per_pass = PirScanQueries(C);
  const int grid = plan.grid;
  ScanArgs a;
  a.db = (const uint4*)db;
  a.sel = (const uint4*)selections;
  a.partials = (uint4*)partials;
  a.num_records = num_records;
  a.sel_blocks = selection_blocks;
  a.C = C;
  a.total_q = num_queries;
  a.parts = grid;
  a.qgroups = 1;
  a.slots = plan.slots ? kScanSlots : 0;
  a.skip = t_scan_skip;
  a.slice_major = 0;
  const dim3 g(grid, (C + 63) / 64);
  for (int q0 = 0; q0 < num_queries;) {
    const int rem = num_queries - q0;
    const bool m4 = !plan.slots && UseScanM4(rem, C);
    const int nq = m4 ? PirScanM4Queries(rem) : std::min(per_pass, rem);
    a.q0 = q0;
    a.nq = nq;
    int rc = m4 ? LaunchPirScanM4(nq, grid, (C + 15) / 16, st, a) : LaunchPirScan(nq, g, st, a);
    if (rc != DPF_AMD_OK) return rc;
    q0 += nq;
  }
  return DPF_AMD_OK;
}

int ExpandBatched(int64_t num_keys, const void* root_seeds, const uint8_t* root_cb,
                  int num_levels, const void* correction_seeds, const uint8_t* ccl,
                  const uint8_t* ccr, const dpf_amd_value_type* vt, const void* key_corr,
                  const int8_t* key_party, int cepb, int64_t leaf_begin, int64_t leaf_end,
                  void* out, void* stream) {
  if (num_keys <= 0 || leaf_end <= leaf_begin) return DPF_AMD_OK;
  if (!vt || num_levels < 11 || num_levels > 62 || leaf_begin < 0 ||
      leaf_end > (int64_t{1} << num_levels))
    return SetError(DPF_AMD_INVALID_ARGUMENT, "bad batched expansion");
  VtDev dev;
  int rc = MakeVtDev(*vt, nullptr, 0, cepb, &dev);
  if (rc != DPF_AMD_OK) return rc;
  if (!SingleDirect(dev))
    return SetError(DPF_AMD_UNIMPLEMENTED, "batched expansion needs a directly convertible type");
  const int64_t range = leaf_end - leaf_begin;
  int D = BatchedDepth(num_keys, range, dev.sc[0].bytes == 16);
  const int forced = t_expand_depth;
  if (forced > 0 && forced <= num_levels) D = forced;
  if (forced < 0) D = forced;
  if (D > num_levels) D = 4;
  const int sub = CoopSub(D);
  ExpandArgs a{};
  a.root_seeds = (const uint4*)root_seeds;
  a.root_cb = root_cb;
  a.cw_seed = (const uint4*)correction_seeds;
  a.ccl = ccl;
  a.ccr = ccr;
  a.out = (char*)out;
  a.walk = num_levels - sub;
  a.chunk_begin = leaf_begin >> sub;
  a.chunk_end = (leaf_end + (1ll << sub) - 1) >> sub;
  a.leaf_begin = leaf_begin;
  a.leaf_end = leaf_end;
  a.batched = 1;
  a.num_levels = num_levels;
  a.num_keys = num_keys;
  a.key_out_stride = range * cepb * dev.stride;  // single direct: stride = element bytes
  a.key_corr = (const uint4*)key_corr;
  a.key_party = key_party;
  return LaunchExpandForType(D, 1, (hipStream_t)stream, a, dev);
}

int PackedCorrection(const dpf_amd_value_type& vt, const uint64_t* correction, int cepb,
                     uint64_t out[2]) {
  VtDev dev;
  const int rc = MakeVtDev(vt, correction, 0, cepb, &dev);
  if (rc != DPF_AMD_OK) return rc;
  out[0] = (uint64_t)dev.corr_packed;
  out[1] = (uint64_t)(dev.corr_packed >> 64);
  return DPF_AMD_OK;
}

int EvaluatePointsBatchedRange(int64_t num_keys, int64_t first_point, int64_t points_per_key,
                               const void* key_seeds, const uint8_t* key_control_bits,
                               int num_levels, const void* correction_seeds, const uint8_t* ccl,
                               const uint8_t* ccr, const dpf_amd_value_type* vt,
                               const int8_t* key_party, const void* key_value_corrections,
                               void* out, void* stream) {
  if (num_keys < 0 || points_per_key < 0 || first_point < 0)
    return SetError(DPF_AMD_INVALID_ARGUMENT, "bad point range");
  if (num_keys > 0 && points_per_key > INT64_MAX / num_keys)
    return SetError(DPF_AMD_INVALID_ARGUMENT, "too many points");
  if (num_keys == 0 || points_per_key == 0) return DPF_AMD_OK;
  return EvaluatePoints(num_keys * points_per_key, points_per_key, num_keys * num_levels,
                        key_seeds, key_control_bits, nullptr, 0, num_levels, correction_seeds,
                        ccl, ccr, vt, nullptr, key_party, 0, key_value_corrections, nullptr, out,
                        nullptr, nullptr, stream, first_point);
}

int EvaluatePointsIndexed(int64_t num_points, const int32_t* key_index, int64_t num_keys,
                          const void* seeds, const uint8_t* control_bits, bool seeds_by_key,
                          const void* paths, int paths_rightshift, int num_levels,
                          const void* correction_seeds, const uint8_t* ccl, const uint8_t* ccr,
                          const dpf_amd_value_type* vt, const uint8_t* block_index,
                          const int8_t* key_party, const void* key_value_corrections, void* out,
                          void* seeds_out, uint8_t* control_bits_out, void* stream) {
  if (num_points < 0 || num_keys < 0 || !key_index)
    return SetError(DPF_AMD_INVALID_ARGUMENT, "bad indexed point evaluation");
  if (num_points == 0) return DPF_AMD_OK;
  return EvaluatePoints(num_points, 0, num_keys * num_levels, seeds, control_bits, paths,
                        paths_rightshift, num_levels, correction_seeds, ccl, ccr, vt, block_index,
                        key_party, 0, key_value_corrections, nullptr, out, seeds_out,
                        control_bits_out, stream, 0, key_index, seeds_by_key);
}
}  // namespace dpf_amd

extern "C" {

int dpf_amd_dcf_evaluate(int64_t num_keys, const void* seeds, const uint8_t* control_bits,
                         const int8_t* party, const void* points, int log_domain_size,
                         const int32_t* tree_level_of, const void* correction_seeds,
                         const uint8_t* ccl, const uint8_t* ccr, const dpf_amd_value_type* vt,
                         const void* value_corrections, void* out, void* stream) {
  if (num_keys < 0 || !vt || !tree_level_of)
    return SetError(DPF_AMD_INVALID_ARGUMENT, "bad arguments");
  if (log_domain_size < 1 || log_domain_size > kDcfMaxLevels)
    return SetError(DPF_AMD_INVALID_ARGUMENT, "A DCF must have log_domain_size >= 1");
  for (int h = 0; h < log_domain_size; ++h)
    if (tree_level_of[h] < 0 || tree_level_of[h] > h ||
        (h > 0 && tree_level_of[h] < tree_level_of[h - 1]))
      return SetError(DPF_AMD_INVALID_ARGUMENT, "invalid hierarchy-to-tree map");
  if (num_keys == 0) return DPF_AMD_OK;
  VtDev dev;
  int rc = MakeVtDev(*vt, nullptr, 0, vt->elements_per_block, &dev);
  if (rc != DPF_AMD_OK) return rc;
  DcfArgs a;
  a.n = num_keys;
  a.seeds = (const uint4*)seeds;
  a.cb = control_bits;
  a.party = party;
  a.points = (const uint4*)points;
  a.cw_seed = (const uint4*)correction_seeds;
  a.ccl = ccl;
  a.ccr = ccr;
  a.corrections = (const uint4*)value_corrections;
  a.out = (char*)out;
  a.log_domain = log_domain_size;
  for (int h = 0; h < kDcfMaxLevels; ++h) a.tree_of[h] = h < log_domain_size ? tree_level_of[h] : 0;
  return LaunchDcfEvaluate(BnTemplate(dev.bn), (hipStream_t)stream, a, dev);
}

int dpf_amd_gather_rows(int64_t num_prefixes, const int64_t* src_offset,
                        int64_t outputs_per_prefix, int64_t stride, const void* in, void* out,
                        void* stream) {
  if (num_prefixes <= 0 || outputs_per_prefix <= 0) return DPF_AMD_OK;
  const int64_t total = num_prefixes * outputs_per_prefix * stride;
  return LaunchGatherRows(GridFor(total, 256, 8192), (hipStream_t)stream, num_prefixes,
                          src_offset, outputs_per_prefix, stride, (const char*)in, (char*)out);
}

int dpf_amd_gather_rows_checked(int64_t num_prefixes, const int64_t* src_offset,
                                int64_t outputs_per_prefix, int64_t stride, const void* in,
                                int64_t in_rows, void* out, int* err, void* stream) {
  if (num_prefixes <= 0 || outputs_per_prefix <= 0) return DPF_AMD_OK;
  const int64_t total = num_prefixes * outputs_per_prefix * stride;
  return LaunchGatherRows(GridFor(total, 256, 8192), (hipStream_t)stream, num_prefixes,
                          src_offset, outputs_per_prefix, stride, (const char*)in, (char*)out,
                          in_rows, err);
}

int dpf_amd_xor_fold(const void* parts, int num_parts, int64_t bytes, void* out,
                     void* stream) {
  if (num_parts <= 0 || bytes <= 0) return DPF_AMD_OK;
  hipStream_t st = (hipStream_t)stream;
  if (bytes % 16 == 0 && ((uintptr_t)parts % 16 == 0) && ((uintptr_t)out % 16 == 0)) {
    const int64_t words = bytes / 16;
    const int64_t blocks = (words + kFoldWords - 1) / kFoldWords;
    if (blocks > INT32_MAX) return SetError(DPF_AMD_INVALID_ARGUMENT, "xor fold too large");
    return LaunchXorFold((unsigned)blocks, st, (const uint4*)parts, num_parts, words,
                         (uint4*)out);
  }
  return LaunchXorFoldBytes(GridFor(bytes, 256, 4096), st, (const uint8_t*)parts, num_parts,
                            bytes, (uint8_t*)out);
}

int64_t dpf_amd_inner_product_workspace_size(int64_t num_records, int64_t record_stride,
                                             int num_queries) {
  return (int64_t)ScanGrid(num_records, num_queries, record_stride) * num_queries *
         record_stride;
}

int dpf_amd_inner_product(const void* db, int64_t num_records, int64_t record_stride,
                          const void* selections, int64_t selection_blocks, int num_queries,
                          void* workspace, void* out, void* stream) {
  if (num_queries == 0) return DPF_AMD_OK;
  const dpf_amd::ScanPlan plan = dpf_amd::PlanScan(num_records, record_stride, num_queries);
  hipStream_t st = (hipStream_t)stream;
  if (plan.slots) {
    int rc = HipCheck(hipMemsetAsync(workspace, 0, dpf_amd::ScanFoldParts(plan) *
                                                       (int64_t)num_queries * record_stride,
                                     st),
                      "scan slots memset");
    if (rc != DPF_AMD_OK) return rc;
  }
  int rc = dpf_amd::ScanPiece(db, num_records, record_stride, selections, selection_blocks,
                              num_queries, plan, workspace, stream);
  if (rc != DPF_AMD_OK) return rc;
  return dpf_amd_xor_fold(workspace, dpf_amd::ScanFoldParts(plan),
                          (int64_t)num_queries * record_stride, out, stream);
}

}  // extern "C"