// internal.h — helpers shared by the HIP kernels and the C++ host library.
#pragma once

#include <stdint.h>

#include <string>

#include "aes_tables.h"
#include "dpf_amd.h"

namespace dpf_amd {

// Thread-local error message for dpf_amd_last_error().
int SetError(int code, const std::string& message);
const char* LastError();

// Idle per-thread resource objects kept per kind (dpf_amd_set_thread_cache_cap).
int ThreadCacheCap();
// dpf_amd_set_force_peer_copies: cross-device copy branches on one device.
bool ForcePeerCopies();
// dpf_amd_set_prefix_expand / DPF_AMD_PREFIX_EXPAND=0: EvaluateUntil expands
// unique tree indices and gathers, instead of expanding per prefix.
bool PrefixExpandOff();
// dpf_amd_set_prefix_expand(2) / DPF_AMD_HOST_INCREMENTAL=1: EvaluateUntil
// keeps the prefix de-duplication, the lookup of the stored partial
// evaluations and the context on the host (the device path's A/B).
bool HostIncremental();

// Device-side copy of dpf_amd_value_type plus everything the per-leaf
// correction needs (kernel argument, < 2 KiB).
constexpr int kMaxScalars = DPF_AMD_MAX_SCALARS;
constexpr int kMaxCorrections = DPF_AMD_MAX_CORRECTIONS;

struct alignas(16) ScalarDev {
  int32_t kind;
  int32_t bytes;
  int32_t in_off;
  int32_t out_off;
  int32_t fold_w;    // IntModN fast reduction: m = 2^fold_w - fold_c
  int32_t use_fold;  // 1 if the folding reduction is used
  int32_t pad0, pad1;
  u128 mod;
  u128 fold_c;
};

struct alignas(16) VtDev {
  int32_t ns;
  int32_t direct;
  int32_t epb;
  int32_t esz;
  int32_t bn;
  int32_t stride;
  int32_t cepb;
  int32_t party;
  ScalarDev sc[kMaxScalars];
  u128 corr[kMaxCorrections];  // [element][scalar]
  u128 corr_packed;  // single-scalar direct types: corrections packed like a block
};

// Stream-ordered copy of `bytes` from host memory mapped into the device
// address space (hipHostMalloc) to device memory, done by a kernel on
// `stream` (host_device.h UploadRing).
int CopyFromMappedHost(void* dst, const void* mapped_src, size_t bytes, void* stream);

// Fills the device descriptor; returns a status code.
int MakeVtDev(const dpf_amd_value_type& vt, const uint64_t* correction,
              int party, int cepb, VtDev* out);

// Full-domain expansion of leaves [leaf_begin, leaf_end) of each of
// num_keys keys of one single-scalar directly convertible type in one
// launch (KExpandCoop, batched): root_seeds / root_cb [key], correction
// words [key][level], key_corr [key] (PackedCorrection), key_party [key];
// key k's outputs at out + k * (leaf_end - leaf_begin) * cepb * out_stride.
// Needs num_levels >= 11.  Device pointers, stream-ordered.
int ExpandBatched(int64_t num_keys, const void* root_seeds, const uint8_t* root_cb,
                  int num_levels, const void* correction_seeds, const uint8_t* ccl,
                  const uint8_t* ccr, const dpf_amd_value_type* vt, const void* key_corr,
                  const int8_t* key_party, int cepb, int64_t leaf_begin, int64_t leaf_end,
                  void* out, void* stream);
// The value correction of a single-scalar direct type packed like one hashed
// block (the form KExpand's EmitDirect adds), for ExpandBatched's key_corr.
int PackedCorrection(const dpf_amd_value_type& vt, const uint64_t* correction, int cepb,
                     uint64_t out[2]);

// dpf_amd_evaluate_points_batched with implicit paths over the tree-index
// range [first_point, first_point + points_per_key) of every key (the leaf
// range of a batched selection expansion on one shard of a database).
int EvaluatePointsBatchedRange(int64_t num_keys, int64_t first_point, int64_t points_per_key,
                               const void* key_seeds, const uint8_t* key_control_bits,
                               int num_levels, const void* correction_seeds, const uint8_t* ccl,
                               const uint8_t* ccr, const dpf_amd_value_type* vt,
                               const int8_t* key_party, const void* key_value_corrections,
                               void* out, void* stream);

// Point evaluation where point i belongs to key key_index[i] of num_keys
// (EvaluateAndApply over key pointers with repeats): correction words
// [key][level], key_party / key_value_corrections per key; starting seeds
// per key (seeds_by_key) or per point.  Device pointers, stream-ordered.
int EvaluatePointsIndexed(int64_t num_points, const int32_t* key_index, int64_t num_keys,
                          const void* seeds, const uint8_t* control_bits, bool seeds_by_key,
                          const void* paths, int paths_rightshift, int num_levels,
                          const void* correction_seeds, const uint8_t* ccl, const uint8_t* ccr,
                          const dpf_amd_value_type* vt, const uint8_t* block_index,
                          const int8_t* key_party, const void* key_value_corrections, void* out,
                          void* seeds_out, uint8_t* control_bits_out, void* stream);

// EvaluateUntil's per-prefix roots in one launch: prefix i starts from row
// idx[i] of seeds / cb (the context walk's output) and walks `walk` (< 8)
// levels along the bits of low[i] with the DPF keys and correction words
// [level] (cw_seed / ccl / ccr).  Device pointers, stream-ordered.
int PrefixRoots(int64_t n, const int32_t* idx, const uint8_t* low, int walk, int64_t num_src,
                const void* seeds, const uint8_t* cb, const void* cw_seed, const uint8_t* ccl,
                const uint8_t* ccr, void* seeds_out, uint8_t* cb_out, void* stream);

// EvaluateUntil's prefix bookkeeping on the device (k_incremental.hip).
// DedupPrefixes: n (< 2^31) sorted 128-bit prefixes -> their unique tree
// indices p >> bbits in order (`unique`, *count of them), prefix i's unique
// index pidx[i] and low bits plow[i] = p & (2^bbits - 1); *flags |= 1 when
// the prefixes are not sorted, 2 when one is >= limit ({lo, hi}; none when
// null).  block_scratch holds DedupBlocks(n) int64.  LookupPartialEvaluations:
// unique index u < min(*count, n_max) -> the stored partial evaluation of
// unique[u] >> shift (binary search of the strictly increasing stored list)
// or, from_root, the key's root seed / control bit; *flags |= 4 when one is
// missing.  Device pointers, stream-ordered.
int64_t DedupBlocks(int64_t n);
int DedupPrefixes(const void* prefixes, int64_t n, int bbits, const uint64_t* limit,
                  int32_t* pidx, uint8_t* plow, void* unique, int64_t* count,
                  int64_t* block_scratch, int* flags, void* stream);
int LookupPartialEvaluations(const void* unique, const int64_t* count, int64_t n_max, int shift,
                             const void* stored, int64_t stored_n, const void* stored_seeds,
                             const uint8_t* stored_cb, const uint64_t root_seed[2], int root_cb,
                             bool from_root, void* seeds_out, uint8_t* cb_out, int* flags,
                             void* stream);

// Dense-PIR scan of one database piece, split from its fold so several
// pieces on one device can share one workspace and one fold
// (dpf_amd_inner_product = PlanScan + [slot memset] + ScanPiece + fold).
// With `slots` every block XORs its partial atomically into one of
// kScanSlots partials (the workspace must be zeroed first; pieces may share
// the slots); otherwise block b writes partial b of `partials`.  The fold
// then reads ScanFoldParts(plan) partials of num_queries x record_stride
// bytes.  Device pointers, stream-ordered.
struct ScanPlan {
  int grid = 1;
  bool slots = false;
};
ScanPlan PlanScan(int64_t num_records, int64_t record_stride, int num_queries);
int ScanFoldParts(const ScanPlan& plan);
int ScanPiece(const void* db, int64_t num_records, int64_t record_stride,
              const void* selections, int64_t selection_blocks, int num_queries,
              const ScanPlan& plan, void* partials, void* stream);
// dpf_amd_xor_fold that leaves the parts zeroed (fold slots reused by the
// next request without a memset).
int XorFoldClear(void* parts, int num_parts, int64_t bytes, void* out, void* stream);

}  // namespace dpf_amd
