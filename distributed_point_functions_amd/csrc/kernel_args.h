// kernel_args.h — POD argument blocks of the gfx950 kernels and the host
// launchers each kernel translation unit exports (the kernels are split over
// several .hip files so hipcc compiles them in parallel).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <string>

#include "aes_tables.h"
#include "internal.h"

namespace dpf_amd {

constexpr int kTabWords = 256 * 64;  // 64 KiB
constexpr int kBlock = 256;  // 64 KiB LDS table per block; 2 blocks per CU
#ifndef DPF_EXPAND_BLOCK
#define DPF_EXPAND_BLOCK 768
#define DPF_EXPAND_WAVES 6
#endif
// KExpand: threads per block and the minimum waves per SIMD the register
// allocation must allow.  Two blocks per CU (one 64 KiB table each) = 24
// waves/CU = 6 per SIMD: the T-table reads need several waves per SIMD to
// keep the LDS busy (measured: 2 waves/SIMD 19.4, 4: 23.6, 6: 24.0 G leaves/s
// on c5; 8 waves spill more and gain nothing).
constexpr int kExpandBlock = DPF_EXPAND_BLOCK;
constexpr int kExpandWaves = DPF_EXPAND_WAVES;

struct KeyPair {
  AesKey k[2];
};

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
  // Non-batched KExpand with precomputed roots: root_seeds are the tree nodes
  // root_level levels below the key's root (root_seeds[i] = node root_base +
  // i of that level), so chunk c starts at root_seeds[(c >> walk) -
  // root_base] and walks levels root_level .. root_level + walk - 1.
  // root_cb == nullptr: the control bit is the seed's LSB (packed nodes).
  int32_t root_level;
  int64_t root_base;
  // Batched keys (KExpandCoop<.., true>): key k = blockIdx.x / (chunk_end -
  // chunk_begin) has root_seeds[k] / root_cb[k], correction words
  // [k * num_levels + level], value correction key_corr[k] (packed block of
  // a single-scalar direct type) and party key_party[k]; the leaf range is
  // per key and key k's outputs start at out + k * key_out_stride bytes.
  int32_t batched;
  int32_t num_levels;
  int64_t num_keys;
  int64_t key_out_stride;
  const uint4* key_corr;
  const int8_t* key_party;
};

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
  // > 0: batched keys — point i belongs to key i / points_per_key; seeds_in,
  // cb_in, party and value_corrections are per key and the correction words
  // are [key][level].  0: per-seed / shared correction words (num_cw).
  int64_t points_per_key;
  int32_t num_levels;
  int32_t rightshift;
  // implicit paths (paths == nullptr): point j of each key walks tree index
  // path_offset + j (a leaf range of a batched selection expansion)
  int64_t path_offset;
  // Non-null: point i belongs to key key_index[i] (EvaluateAndApply over a
  // span of key pointers with repeats); correction words [key][level],
  // party and value corrections per key.  The walk's starting seeds are per
  // key when seeds_by_key, else per point (a later hierarchy level resumes
  // from the previous level's per-point seeds).
  const int32_t* key_index;
  int32_t seeds_by_key;
  int32_t pad;
};

struct PointsArgs {
  WalkArgs w;
  const uint8_t* block_index;
  const int8_t* party;
  const uint4* value_corrections;  // per seed: epb * ns 128-bit words
  char* out;
};

// KDcfEvaluate (dcf/distributed_comparison_function.h:141-187): key i at
// point i, hierarchy level h has log domain h (h < log_domain), rightshift 1.
constexpr int kDcfMaxLevels = 128;
struct DcfArgs {
  int64_t n;
  const uint4* seeds;
  const uint8_t* cb;
  const int8_t* party;
  const uint4* points;
  const uint4* cw_seed;  // [tree level][key]
  const uint8_t* ccl;
  const uint8_t* ccr;
  const uint4* corrections;  // [hierarchy level][key][epb * ns]
  char* out;
  int32_t log_domain;  // DCF log domain = number of hierarchy levels
  int32_t tree_of[kDcfMaxLevels];  // hierarchy level -> tree level
};

// KEvaluatePoints: 2 blocks per CU (one 64 KiB table each), 4 waves/SIMD,
// two points per thread walked in lockstep.
#ifndef DPF_POINTS_BLOCK
#define DPF_POINTS_BLOCK 512
#define DPF_POINTS_WAVES 4
#endif
constexpr int kPointsBlock = DPF_POINTS_BLOCK;
constexpr int kPointsWaves = DPF_POINTS_WAVES;

constexpr int kScanBlock = 256;
constexpr int kScanWaves = kScanBlock / 64;
constexpr int kFoldWords = 4;
constexpr int kFoldSlices = 64;

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
  int32_t parts;        // partials written per query (KPirScanM4: waves in use)
  int32_t qgroups;      // KPirScanM4: waves scanning the same tiles (1 or 2)
  // KPirScanG: 0 = one partial per block; S > 0 = block b XORs its partial
  // atomically into partial slot b % S (zeroed before the scan), so the fold
  // reads S partials instead of one per block.
  int32_t slots;
  // KPirScanG (records of 32 B and more): 0 (default) = every record is
  // read, an access pattern independent of the selection; 1 (opt-in,
  // DPF_AMD_SCAN_SKIP_UNSELECTED=1) = a record no query of the pass selects
  // is not read, as the reference's scan skips it (inner_product_hwy.cc:
  // 213-221) — the access pattern then follows the selection share.
  int32_t skip;
  // KPirScanM4*: 1 = a 1-D grid of (part block, 256-byte slice) pairs,
  // slice-major and XCD-local (set by LaunchPirScanM4)
  int32_t slice_major;
};

// Fold slots of the masked scan when a pass's partial is small: 64 slots,
// for at most kScanSlotMaxBytes of partial (queries x record bytes) per block.
constexpr int kScanSlots = 64;
constexpr int64_t kScanSlotMaxBytes = 2048;

// KPirScanM4: 4 independent waves per block, one LDS table pair per wave.
constexpr int kScanM4Block = 256;
constexpr int kScanM4Waves = kScanM4Block / 64;
// Queries from which a scan pass uses KPirScanM4 (records of >= 64 bytes).
// c4 (2^26 x 256 B), round 5 (profiles/c4q_masked_vs_m4_r05.log): Q = 8
// masked 2.60 ms vs M4 2.84; Q = 9 2.86 vs 2.64, 12 2.96 vs 2.66, 15 3.12 vs
// 2.69 (round 2 had measured only Q = 8 and 16 and set the switch at 16).
#ifndef DPF_AMD_SCAN_M4_MIN_Q
#define DPF_AMD_SCAN_M4_MIN_Q 9
#endif
constexpr int kScanM4MinQueries = DPF_AMD_SCAN_M4_MIN_Q;

inline int HipCheck(hipError_t e, const char* what) {
  if (e == hipSuccess) return DPF_AMD_OK;
  const int code =
      (e == hipErrorOutOfMemory) ? DPF_AMD_RESOURCE_EXHAUSTED : DPF_AMD_INTERNAL;
  return SetError(code, std::string(what) + ": " + hipGetErrorString(e));
}

inline int LaunchCheck(const char* what) { return HipCheck(hipGetLastError(), what); }


// k_expand_nodes.hip: the 1024-node levels of blocks [chunk_begin, chunk_end)
// as packed nodes (KExpandCoop<0, EmitNodes>).
int LaunchExpandNodes(hipStream_t st, const ExpandArgs& a, const VtDev& vt);
// k_expand_*.hip: fused expansion with DFS depth D in {0,1,2,4,8}.
int LaunchExpandU32ModN64(int D, int grid, hipStream_t st, const ExpandArgs& a,
                          const VtDev& vt);
int LaunchExpandDirect1(int D, int grid, hipStream_t st, const ExpandArgs& a, const VtDev& vt);
int LaunchExpandDirect2(int D, int grid, hipStream_t st, const ExpandArgs& a, const VtDev& vt);
int LaunchExpandDirect4(int D, int grid, hipStream_t st, const ExpandArgs& a, const VtDev& vt);
int LaunchExpandDirect8(int D, int grid, hipStream_t st, const ExpandArgs& a, const VtDev& vt);
int LaunchExpandDirect16(int D, int grid, hipStream_t st, const ExpandArgs& a, const VtDev& vt);
int LaunchExpandGeneric1(int D, int grid, hipStream_t st, const ExpandArgs& a, const VtDev& vt);
int LaunchExpandGeneric2(int D, int grid, hipStream_t st, const ExpandArgs& a, const VtDev& vt);
int LaunchExpandGeneric4(int D, int grid, hipStream_t st, const ExpandArgs& a, const VtDev& vt);
// k_walk.hip
int LaunchEvaluateSeeds(int64_t n, hipStream_t st, const WalkArgs& a, const KeyPair& kp);
int LaunchEvaluateSeedsDpf(int64_t n, hipStream_t st, const WalkArgs& a, const KeyPair& kp);
int LaunchEvaluatePoints(int bn, int64_t n, hipStream_t st, const PointsArgs& a,
                         const VtDev& vt);
// The calling thread's point-walk kernel choice (dpf_amd_set_walk_mode).
int WalkMode();
// Whether this thread's DCF launches may use the single-scalar kernel
// (dpf_amd_set_dcf_kernel).
bool DcfDirectEnabled();
int LaunchDcfEvaluate(int bn, hipStream_t st, const DcfArgs& a, const VtDev& vt);
int LaunchAesMmo(int grid, hipStream_t st, const uint4* in, uint4* out, int64_t n,
                 const KeyPair& kp);
// k_pir.hip
int LaunchGatherRows(int grid, hipStream_t st, int64_t n, const int64_t* src_offset,
                     int64_t opp, int64_t stride, const char* in, char* out,
                     int64_t in_rows = INT64_MAX, int* err = nullptr);
int LaunchXorFold(unsigned blocks, hipStream_t st, const uint4* parts, int num_parts,
                  int64_t words, uint4* out, uint4* clear = nullptr);
int LaunchXorFoldBytes(int grid, hipStream_t st, const uint8_t* parts, int num_parts,
                       int64_t bytes, uint8_t* out);
int LaunchPirScan(int nq, dim3 grid, hipStream_t st, const ScanArgs& a);
// Records per wave-instruction of KPirScanG for C chunks per record;
// queries per scan pass = PirScanQueries(C).
int PirScanGroup(int C);
inline int PirScanQueries(int) { return 16; }
// Four-Russians scan: queries of the next pass (of `rem` left), and the
// launch of one pass of nq <= PirScanM4Queries(nq) queries over `slices`
// 256-byte column slices of the record, writing `parts` partials per query.
int PirScanM4Queries(int rem);
int LaunchPirScanM4(int nq, int parts, int slices, hipStream_t st, const ScanArgs& a);

}  // namespace dpf_amd

// The T-table fill (aes_device.h FillRows) gives each wave whole table rows:
// every block that fills tables has a multiple of 64 threads, at most 1024
// (the run-time block sizes, WalkBlock and the quad launch, round to 64).
static_assert(dpf_amd::kExpandBlock % 64 == 0 && dpf_amd::kExpandBlock <= 1024,
              "expansion blocks must be whole waves");
static_assert(dpf_amd::kPointsBlock % 64 == 0 && dpf_amd::kPointsBlock <= 1024,
              "walk blocks must be whole waves");
