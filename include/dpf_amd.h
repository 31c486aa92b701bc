/*
 * dpf_amd.h — C ABI of the MI355X-native DPF / dense-PIR hot path.
 *
 * Every entry point is `extern "C"`, takes plain pointers and sizes (no torch,
 * no C++ types), and returns an int status equal to the absl::StatusCode
 * number the reference would return (0 OK, 3 INVALID_ARGUMENT, 8
 * RESOURCE_EXHAUSTED, 9 FAILED_PRECONDITION, 12 UNIMPLEMENTED, 13 INTERNAL).
 * The message of the last failure on the calling thread is returned by
 * dpf_amd_last_error().
 *
 * 128-bit integers (absl::uint128 in the reference) cross the ABI as two
 * little-endian 64-bit words {lo, hi} — the in-memory layout of
 * absl::uint128 / unsigned __int128 on x86-64 — so arrays of them are
 * interchangeable with the reference's `absl::uint128*`.
 *
 * Two tiers:
 *   Tier 1 (device pointers, stream-ordered): the internal seams of the
 *     reference's hot path that the HIP kernels replace.  Inputs and outputs
 *     live in HBM; `stream` is a hipStream_t (NULL = default stream).
 *   Tier 2 (host memory, opaque handles): the reference's public objects
 *     (DistributedPointFunction, EvaluationContext, DenseDpfPirServer) with
 *     DpfKey / EvaluationContext / PirRequest / PirResponse exchanged in
 *     protobuf wire format, exactly as a cgo / JNI / ctypes binding of the
 *     reference would pass them.
 * Reference file:line citations use the paths under /root/reference.
 */
#ifndef DPF_AMD_H_
#define DPF_AMD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DPF_AMD_OK 0
#define DPF_AMD_INVALID_ARGUMENT 3
#define DPF_AMD_RESOURCE_EXHAUSTED 8
#define DPF_AMD_FAILED_PRECONDITION 9
#define DPF_AMD_UNIMPLEMENTED 12
#define DPF_AMD_INTERNAL 13

#define DPF_AMD_MAX_SCALARS 16
#define DPF_AMD_MAX_CORRECTIONS 32
#define DPF_AMD_MAX_BLOCKS_NEEDED 4

/* Kinds are the proto field numbers of ValueType's oneof
 * (dpf/distributed_point_function.proto:25-60). */
#define DPF_AMD_KIND_INTEGER 1
#define DPF_AMD_KIND_INT_MOD_N 3
#define DPF_AMD_KIND_XOR_WRAPPER 4

/* One scalar of a (flattened) value type T. */
typedef struct {
  int32_t kind;        /* DPF_AMD_KIND_* */
  int32_t bytes;       /* sizeof(scalar): 1, 2, 4, 8 or 16 */
  int32_t in_offset;   /* byte offset inside one element when converted
                          directly (ValueTypeHelper::DirectlyFromBytes) */
  int32_t out_offset;  /* byte offset inside one host-layout T */
  uint64_t modulus[2]; /* IntModN modulus {lo, hi}; 0 otherwise */
} dpf_amd_scalar;

/* Runtime description of the value type T of EvaluateUntil<T> /
 * EvaluateAt<T> — the template parameter cannot cross a C ABI, so the host
 * passes what the reference's header templates compute at compile time
 * (h:816-862, vth:525-606).  Produced by dpf_amd_describe_value_type(). */
typedef struct {
  int32_t num_scalars;
  int32_t directly_convertible; /* can_be_converted_directly_v<T> */
  int32_t elements_per_block;   /* ElementsPerBlock<T>() */
  int32_t element_size;         /* (TotalBitSize<T>() + 7) / 8 (direct only) */
  int32_t blocks_needed;        /* ceil(BitsNeeded / 128) (cc:603-610) */
  int32_t out_stride;           /* sizeof(T) in the host layout */
  int32_t reserved[2];
  dpf_amd_scalar scalars[DPF_AMD_MAX_SCALARS];
} dpf_amd_value_type;

const char* dpf_amd_last_error(void);

/* Library / device info.  dpf_amd_version ends in "src:<sha256>", the hash
 * of the sources and build flags the library was compiled from. */
int dpf_amd_device_count(int* count);
const char* dpf_amd_version(void);
/* Returns the idle device blocks the library's caching allocator holds to
 * the device (a caller about to make a large allocation of its own, e.g. a
 * database or a torch tensor, after Tier-2 calls left blocks cached); writes
 * the bytes released to *released (may be NULL). */
int dpf_amd_release_cached_memory(int64_t* released);

/* Per-thread host resources (streams, pinned staging, incremental scratch)
 * outlive their thread in a process-wide free list, so a server answering
 * from short-lived threads creates them once per concurrent thread.  At most
 * `cap` idle objects of each kind are kept (default 64, or
 * DPF_AMD_THREAD_CACHE); the surplus is destroyed by the next thread that
 * takes one, never in a thread-exit handler. */
int dpf_amd_set_thread_cache_cap(int cap);

/* Test hook (process-wide): 1 = a sharded DenseDpfPirDatabase takes the
 * cross-device branches even between shards on one device (hipMemcpyPeer
 * of the rows in Build, hipMemcpyPeerAsync of the partials in the combine),
 * so one GPU executes the code an 8-GPU node runs.  0 = automatic. */
void dpf_amd_set_force_peer_copies(int on);

/* ------------------------------------------------------------------------ */
/* Tier 1: device seams                                                     */
/* ------------------------------------------------------------------------ */

/* Replaces Aes128FixedKeyHash::Evaluate (dpf/aes_128_fixed_key_hash.h:52-53,
 * .cc:57-98): out[i] = AES_key(sigma(in[i])) ^ sigma(in[i]),
 * sigma(x) = (x.hi ^ x.lo, x.hi).  In-place safe. */
int dpf_amd_aes128_mmo(uint64_t key_lo, uint64_t key_hi, const void* in,
                       void* out, int64_t n, void* stream);

/* Replaces dpf_internal::EvaluateSeeds (dpf/internal/evaluate_prg_hwy.h:70-77,
 * .cc:638-658) with the same argument meaning; `prg_left`/`prg_right` are
 * given by their 128-bit keys.  num_correction_words must be num_levels or
 * num_levels * num_seeds (INVALID_ARGUMENT otherwise, .cc:647-652); with
 * per-seed words, seed i at level l uses word l * num_seeds + i.  All arrays
 * are device pointers; seeds_out / control_bits_out may alias the inputs. */
int dpf_amd_evaluate_seeds(int64_t num_seeds, int num_levels,
                           int64_t num_correction_words, const void* seeds_in,
                           const uint8_t* control_bits_in, const void* paths,
                           int paths_rightshift, const void* correction_seeds,
                           const uint8_t* correction_controls_left,
                           const uint8_t* correction_controls_right,
                           uint64_t key_left_lo, uint64_t key_left_hi,
                           uint64_t key_right_lo, uint64_t key_right_hi,
                           void* seeds_out, uint8_t* control_bits_out,
                           void* stream);

/* Fused ExpandSeeds (cc:289-372) + HashExpandedSeeds (cc:523-547) + the
 * per-leaf value correction of EvaluateUntil (h:836-862), on a forest of
 * `num_roots` roots each expanded `num_levels` tree levels with the DPF PRG
 * keys (cc:55-60).  The concatenated leaf (tree block) index of root r,
 * block j is g = r * 2^num_levels + j; leaves g in [leaf_begin, leaf_end)
 * are produced, element e (< corrected_elements_per_block) of leaf g being
 * written in host layout at
 *   out + ((g - leaf_begin) * cepb + e) * vt->out_stride.
 * Only the scalars are written: padding bytes of a host layout with holes
 * keep their previous contents (the Tier-2 API clears them first).
 * Correction words for the num_levels levels are device arrays; the value
 * correction (epb * num_scalars words of 128 bits, flattened per element)
 * and the party are host values (h:815-827, 856-858). */
int dpf_amd_expand_and_correct(
    int64_t num_roots, const void* root_seeds, const uint8_t* root_control_bits,
    int num_levels, const void* correction_seeds,
    const uint8_t* correction_controls_left,
    const uint8_t* correction_controls_right, const dpf_amd_value_type* vt,
    const uint64_t* value_correction, int party,
    int corrected_elements_per_block, int64_t leaf_begin, int64_t leaf_end,
    void* out, void* stream);

/* Full-domain expansion of many keys of one DPF in one launch (the selection
 * vectors of a Q-key PIR request, or any batch of EvaluateUntil keys of a
 * single hierarchy level): leaves [leaf_begin, leaf_end) of each key, key k's
 * outputs at out + k * (leaf_end - leaf_begin) * corrected_elements_per_block
 * * out_stride.  Device arrays: root_seeds [key] (128-bit), root control
 * bits [key], correction words [key][level] (seeds 128-bit, ccl, ccr).  Host
 * arrays: value_corrections [key][elements_per_block * num_scalars] 128-bit
 * words, parties [key].  Single-scalar directly convertible types of >= 11
 * tree levels run one KExpand / KExpandCoop grid over all keys; other types
 * one launch per key.  Stream-ordered on `stream`. */
int dpf_amd_expand_and_correct_batched(
    int64_t num_keys, const void* root_seeds, const uint8_t* root_control_bits,
    int num_levels, const void* correction_seeds, const uint8_t* ccl,
    const uint8_t* ccr, const dpf_amd_value_type* vt,
    const uint64_t* value_corrections, const int8_t* parties,
    int corrected_elements_per_block, int64_t leaf_begin, int64_t leaf_end,
    void* out, void* stream);

/* Testing knob (calling thread only): forces the register-DFS depth D of the
 * fused expansion kernel KExpand to 1, 2, 4, 5, 6 or 8 whenever num_levels >= D,
 * or the cooperative kernel KExpandCoop with 1024 (-1), 2048 (-2) or 256 (-3)
 * leaves per block whenever num_levels >= 10 / 11 / 8, so the kernels that
 * other launch sizes select can be checked on small domains.  0 restores the
 * automatic choice.  Returns the previous setting, or -99 for an invalid
 * value (setting unchanged). */
int dpf_amd_set_expand_depth(int depth);

/* Testing knob (calling thread only): the roots stage of large expansions.
 * A KExpand<8> launch normally walks every thread from the key's root down to
 * its 256-leaf subtree; with the roots stage the nodes six levels above the
 * subtree roots are computed once, breadth-first (KExpandCoop), and each
 * thread walks six levels from there.  -1 = automatic (launches of >= 2^28
 * leaves at D = 8 with >= 17 levels above the subtrees), 0 = never, 1 =
 * whenever the launch is eligible regardless of size (tests).  Every thread
 * starts from -1, or 0 with DPF_AMD_EXPAND_ROOTS=0.  Returns the previous
 * setting, or -2 for an invalid mode (unchanged). */
int dpf_amd_set_expand_roots(int mode);

/* Testing knob (calling thread only): which XOR scan dpf_amd_inner_product
 * runs on launches issued by this thread.
 * -1 automatic (the Four-Russians many-query scan from 16 queries on, records
 * of >= 64 bytes; the masked scan otherwise), 0 always the masked scan, 1
 * always the Four-Russians scan.  Every thread starts from DPF_AMD_SCAN_M4
 * (or -1).
 * Returns the previous setting, or -2 for an invalid mode (unchanged). */
int dpf_amd_set_scan_m4(int mode);

/* Opt-in (calling thread only): 1 = the masked XOR scan (dpf_amd_inner_product,
 * InnerProductWith, HandleRequest; records of >= 32 bytes) reads only the
 * records some query of a pass selects, as the reference's InnerProduct
 * skips unselected records (inner_product_hwy.cc:213-221) — about half the
 * table at one query; the scan's memory access pattern then follows the
 * selection share.  0 (the default) = every record is read, an access
 * pattern independent of the selection.  Every thread starts from
 * DPF_AMD_SCAN_SKIP_UNSELECTED (or 0).  Returns the previous setting, or -2
 * for an invalid value (unchanged). */
int dpf_amd_set_scan_skip_unselected(int on);

/* Test hook: the calling thread's point-walk kernel (EvaluateAt /
 * EvaluateAndApply / the batched point evaluation).  0 = automatic (four
 * lanes per point below 65,536 points for types of <= 256 bits, one lane per
 * point above), 1 = four lanes per point whenever the type allows, 2 = one
 * lane per point.  Returns the previous setting, or -2 for an invalid mode
 * (unchanged). */
int dpf_amd_set_walk_mode(int mode);

/* Test hook: the calling thread's EvaluateUntil strategy for calls with
 * prefixes.  0 = automatic (each prefix's own subtree expanded straight into
 * the output when this level's tree level is at or below the prefix's
 * depth, with the de-duplication, the lookup of the stored partial
 * evaluations and the context's list kept on the device), 1 = the unique
 * tree indices expanded into a staging buffer and gathered per prefix
 * (h:772-889's shape), 2 = as 0 with that bookkeeping on the host.  Returns
 * the previous setting, or -2 for an invalid mode (unchanged). */
int dpf_amd_set_prefix_expand(int mode);

/* Test hook: the calling thread's DCF BatchEvaluate kernel.  0 = automatic
 * (a single integer / XorWrapper scalar runs the register-only kernel),
 * 1 = the generic kernel for every value type.  Returns the previous
 * setting, or -2 for an invalid mode (unchanged). */
int dpf_amd_set_dcf_kernel(int mode);

/* Fused single-path evaluation: EvaluateSeeds from the given seeds along
 * `paths` (one AES per level, per-lane key select) + HashExpandedSeeds +
 * correction of element block_index[i] (EvaluateAtImpl h:1013-1063 and the
 * per-key loop of EvaluateAndApply h:1143-1189).  Per-seed arrays:
 * seeds, control_bits, paths, block_index (may be NULL = 0), party (NULL =
 * `party_all`), value_corrections (NULL = `value_correction_all`, else
 * num_seeds * epb * num_scalars words).  Correction words are shared
 * (num_cw == num_levels) or per seed (num_levels * num_seeds).  Writes one
 * host-layout T per seed, and optionally the final seeds / control bits. */
int dpf_amd_evaluate_points(
    int64_t num_seeds, const void* seeds, const uint8_t* control_bits,
    const void* paths, int paths_rightshift, int num_levels,
    int64_t num_correction_words, const void* correction_seeds,
    const uint8_t* correction_controls_left,
    const uint8_t* correction_controls_right, const dpf_amd_value_type* vt,
    const uint8_t* block_index, const int8_t* party, int party_all,
    const void* value_corrections, const uint64_t* value_correction_all,
    void* out, void* seeds_out, uint8_t* control_bits_out, void* stream);

/* Batched EvaluateAt over `num_keys` keys of one DPF (the per-key loop a
 * caller of EvaluateAtImpl h:913-1070 runs, as one launch): point
 * i = k * points_per_key + j belongs to key k.  Per-key device arrays:
 * key_seeds, key_control_bits, key_party (NULL = `party_all`),
 * key_value_corrections (epb * num_scalars words per key; NULL =
 * `value_correction_all`), and the correction words laid out [key][level]
 * (num_keys * num_levels each).  Per-point: paths (NULL = point j of each
 * key walks to tree index j: the first points_per_key leaves of every key),
 * block_index (NULL = 0), out (one host-layout T per point). */
int dpf_amd_evaluate_points_batched(
    int64_t num_keys, int64_t points_per_key, const void* key_seeds,
    const uint8_t* key_control_bits, const void* paths, int paths_rightshift,
    int num_levels, const void* correction_seeds,
    const uint8_t* correction_controls_left,
    const uint8_t* correction_controls_right, const dpf_amd_value_type* vt,
    const uint8_t* block_index, const int8_t* key_party, int party_all,
    const void* key_value_corrections, const uint64_t* value_correction_all,
    void* out, void* stream);

/* Fused DistributedComparisonFunction::BatchEvaluate
 * (dcf/distributed_comparison_function.h:141-187 over EvaluateAndApply
 * h:1072-1198 with rightshift 1): key i (seed, control bit, party) is
 * evaluated at points[i] through hierarchy levels h < log_domain_size (log
 * domain h, tree level tree_level_of[h], a host array); the outputs of the
 * levels whose DCF bit (log_domain_size - h - 1) of points[i] is 0 are
 * summed with the value type's + into out[i] (host layout).  Device arrays:
 * correction words [tree level][key] (tree_level_of[log_domain_size-1]
 * levels), value corrections [level][key][epb * num_scalars] 128-bit words.
 * `vt` describes the DCF's value type (same at every level). */
int dpf_amd_dcf_evaluate(int64_t num_keys, const void* seeds,
                         const uint8_t* control_bits, const int8_t* party,
                         const void* points, int log_domain_size,
                         const int32_t* tree_level_of,
                         const void* correction_seeds,
                         const uint8_t* correction_controls_left,
                         const uint8_t* correction_controls_right,
                         const dpf_amd_value_type* vt,
                         const void* value_corrections, void* out,
                         void* stream);

/* Gathers the per-prefix output slices of an incremental evaluation
 * (h:877-889): out[i * opp + k] = in[src_offset[i] + k] for k < opp, rows of
 * `stride` bytes. */
int dpf_amd_gather_rows(int64_t num_prefixes, const int64_t* src_offset,
                        int64_t outputs_per_prefix, int64_t stride,
                        const void* in, void* out, void* stream);

/* As dpf_amd_gather_rows with the source size: segments whose source rows
 * fall outside [0, in_rows) are skipped and *err (device int, may be NULL)
 * is set to 1 instead of reading out of bounds. */
int dpf_amd_gather_rows_checked(int64_t num_prefixes, const int64_t* src_offset,
                                int64_t outputs_per_prefix, int64_t stride,
                                const void* in, int64_t in_rows, void* out, int* err,
                                void* stream);

/* Replaces pir_internal::InnerProduct (pir/internal/inner_product_hwy.h:
 * 38-41) for a database stored with a fixed, 16-byte-aligned record stride:
 * for query q, out[q] = XOR of records r < num_records whose selection bit
 * (bit r % 128 of 128-bit block r / 128 of selections[q]) is set.
 * `selections` holds num_queries * selection_blocks 128-bit blocks,
 * `out` num_queries * record_stride bytes.  `workspace` must hold
 * dpf_amd_inner_product_workspace_size() bytes.  The scan reads every record
 * exactly once with 16-byte loads and applies selections with masks
 * (constant-time; no data-dependent skipping). */
int64_t dpf_amd_inner_product_workspace_size(int64_t num_records,
                                             int64_t record_stride,
                                             int num_queries);
int dpf_amd_inner_product(const void* db, int64_t num_records,
                          int64_t record_stride, const void* selections,
                          int64_t selection_blocks, int num_queries,
                          void* workspace, void* out, void* stream);

/* XOR-folds `num_parts` buffers of `bytes` bytes each (parts contiguous) into
 * out — the local fold after an RCCL all-gather of XOR shares (RCCL has no
 * XOR reduction). */
int dpf_amd_xor_fold(const void* parts, int num_parts, int64_t bytes,
                     void* out, void* stream);

/* ------------------------------------------------------------------------ */
/* Tier 2: reference objects behind opaque handles (host memory)            */
/* ------------------------------------------------------------------------ */

typedef struct dpf_amd_dpf dpf_amd_dpf;
typedef struct dpf_amd_ctx dpf_amd_ctx;
typedef struct dpf_amd_pir_db dpf_amd_pir_db;
typedef struct dpf_amd_pir_server dpf_amd_pir_server;

/* Frees a buffer returned by this library (serialized protos). */
void dpf_amd_free(void* p);

/* Fills `vt` (layout + conversion metadata for T) from a serialized
 * ValueType proto and a security parameter (which decides blocks_needed). */
int dpf_amd_describe_value_type(const uint8_t* value_type_proto, size_t len,
                                double security_parameter,
                                dpf_amd_value_type* vt);

/* DistributedPointFunction::CreateIncremental (h:102-103, cc:589-640);
 * each parameters[i] is a serialized DpfParameters proto. */
int dpf_amd_dpf_create_incremental(const uint8_t* const* parameters,
                                   const size_t* lengths, int num_parameters,
                                   dpf_amd_dpf** out);
void dpf_amd_dpf_destroy(dpf_amd_dpf* dpf);
/* Hierarchy metadata (proto_validator.cc:127-153). */
int dpf_amd_dpf_tree_levels_needed(const dpf_amd_dpf* dpf);
int dpf_amd_dpf_hierarchy_to_tree(const dpf_amd_dpf* dpf, int level);
/* Output element type of hierarchy level `level`. */
int dpf_amd_dpf_value_type(const dpf_amd_dpf* dpf, int level,
                           dpf_amd_value_type* vt);

/* GenerateKeysIncremental (h:258-259, cc:642-710).  betas[i] is a serialized
 * Value proto for level i.  If `seeds` is non-NULL it supplies the two root
 * seeds (4 words) instead of the CSPRNG (for reproducible fixtures only).
 * Keys are returned as serialized DpfKey protos (free with dpf_amd_free). */
/* DistributedPointFunction::RegisterValueType<T>() (h:129-131) by ValueType
 * proto.  GenerateKeys with a Value of a type that is neither a single
 * unsigned integer nor registered returns FAILED_PRECONDITION (cc:567-582). */
int dpf_amd_dpf_register_value_type(dpf_amd_dpf* dpf, const uint8_t* value_type_proto,
                                    size_t len);
int dpf_amd_dpf_generate_keys(dpf_amd_dpf* dpf, uint64_t alpha_lo,
                              uint64_t alpha_hi, const uint8_t* const* betas,
                              const size_t* beta_lengths,
                              const uint64_t* seeds, uint8_t** key0,
                              size_t* key0_len, uint8_t** key1,
                              size_t* key1_len);

/* CreateEvaluationContext (h:278, cc:712-727) from a serialized DpfKey. */
int dpf_amd_ctx_create(const dpf_amd_dpf* dpf, const uint8_t* key,
                       size_t key_len, dpf_amd_ctx** out);
/* Parses / serializes a whole EvaluationContext proto. */
int dpf_amd_ctx_parse(const dpf_amd_dpf* dpf, const uint8_t* data, size_t len,
                      dpf_amd_ctx** out);
int dpf_amd_ctx_serialize(const dpf_amd_ctx* ctx, uint8_t** data, size_t* len);
void dpf_amd_ctx_destroy(dpf_amd_ctx* ctx);
int dpf_amd_ctx_previous_hierarchy_level(const dpf_amd_ctx* ctx);
int dpf_amd_ctx_partial_evaluations_level(const dpf_amd_ctx* ctx);
int64_t dpf_amd_ctx_num_partial_evaluations(const dpf_amd_ctx* ctx);

/* EvaluateUntil<T> (h:319-322, 695-891).  `value_type` is the serialized
 * ValueType of T (checked as in h:709-716).  Writes host-layout T values to
 * `out` (capacity in bytes); *num_outputs receives the element count.  With
 * out == NULL only *num_outputs is computed, after the same validation as an
 * evaluation (arguments, context, and every prefix in range, h:735-745);
 * with out == NULL and out_capacity < 0 the prefixes' range check is left
 * to the evaluation call that follows (the two-call protocol's first call:
 * one pass over a long prefix list instead of two). */
int dpf_amd_evaluate_until(const dpf_amd_dpf* dpf, int hierarchy_level,
                           const uint64_t* prefixes, int64_t num_prefixes,
                           const uint8_t* value_type, size_t value_type_len,
                           dpf_amd_ctx* ctx, void* out, int64_t out_capacity,
                           int64_t* num_outputs);

/* As dpf_amd_evaluate_until, with the outputs left in device memory
 * (`out_device`, HBM) and the work ordered on `stream` (NULL = the calling
 * thread's stream): the MI355X consumer path — no PCIe copy of the
 * outputs.  Returns after the outputs are complete. */
int dpf_amd_evaluate_until_device(const dpf_amd_dpf* dpf, int hierarchy_level,
                                  const uint64_t* prefixes, int64_t num_prefixes,
                                  const uint8_t* value_type, size_t value_type_len,
                                  dpf_amd_ctx* ctx, void* out_device,
                                  int64_t out_capacity, int64_t* num_outputs,
                                  void* stream);

/* One key's full-domain leaves spread over devices (the c5 shape of
 * DistributedPointFunction::ExpandLeavesOnDevices): slice i expands leaves
 * [leaf_begin[i], leaf_end[i]) of the last hierarchy level, in the host
 * layout of its value type, into device memory outs[i] on device
 * devices[i]; all slices run concurrently (one stream per device of the
 * calling thread) and the call returns when all are done. */
int dpf_amd_expand_leaves_on_devices(const dpf_amd_dpf* dpf, const uint8_t* key,
                                     size_t key_len, int num_slices,
                                     const int* devices, const int64_t* leaf_begin,
                                     const int64_t* leaf_end, void* const* outs);

/* EvaluateAt<T>(key, level, points) (h:349-354, 913-1070). */
int dpf_amd_evaluate_at(const dpf_amd_dpf* dpf, const uint8_t* key,
                        size_t key_len, int hierarchy_level,
                        const uint64_t* points, int64_t num_points,
                        const uint8_t* value_type, size_t value_type_len,
                        void* out);

/* EvaluateAt<T>(level, points, ctx) (h:356-378; EvaluateAtImpl h:1000-1011):
 * starts from the partial evaluations stored in `ctx` (from the root when it
 * holds none), walks them to `hierarchy_level`'s tree level, writes the
 * num_points host-layout T values to `out`, and rewrites ctx's partial
 * evaluations (the points' tree indices at `hierarchy_level`) and its
 * previous_hierarchy_level.  Errors: the reference's, including "Prefix not
 * present in ctx.partial_evaluations at hierarchy level <h>". */
int dpf_amd_evaluate_at_ctx(const dpf_amd_dpf* dpf, int hierarchy_level,
                            const uint64_t* points, int64_t num_points,
                            const uint8_t* value_type, size_t value_type_len,
                            dpf_amd_ctx* ctx, void* out);

/* EvaluateAndApply<T, Fn> (h:403-407, 1072-1198): evaluates key i at point
 * i level by level, writing num_keys host-layout T values of level h to
 * out + h * num_keys * sizeof(T); after each level `op(user, h, values of
 * level h, num_keys)` is called (if not NULL) and a return of 0 stops the
 * evaluation, as the reference's `op` returning false. */
typedef int (*dpf_amd_apply_fn)(void* user, int hierarchy_level, const void* values,
                                int64_t num_keys);
int dpf_amd_evaluate_and_apply(const dpf_amd_dpf* dpf,
                               const uint8_t* const* keys,
                               const size_t* key_lengths, int64_t num_keys,
                               const uint64_t* points, int rightshift,
                               const uint8_t* value_type,
                               size_t value_type_len, void* out,
                               dpf_amd_apply_fn op, void* user);

/* DistributedComparisonFunction (dcf/distributed_comparison_function.h:30-
 * 187).  Parameters and keys cross as DcfParameters / DcfKey protos; beta as
 * a Value proto; `seeds` (4 words: seed0 lo, hi, seed1 lo, hi) replaces the
 * CSPRNG for fixtures, NULL = CSPRNG.  BatchEvaluate writes num_keys
 * host-layout T values (T = `value_type`, the DCF's value type). */
typedef struct dpf_amd_dcf dpf_amd_dcf;
int dpf_amd_dcf_create(const uint8_t* parameters, size_t len, dpf_amd_dcf** out);
void dpf_amd_dcf_destroy(dpf_amd_dcf* dcf);
/* Registers a value type with the DCF's DPF (what the DCF's templated
 * GenerateKeys<T> does through ToValue<T>, dcf/distributed_comparison_
 * function.h:57-67). */
int dpf_amd_dcf_register_value_type(dpf_amd_dcf* dcf, const uint8_t* value_type_proto,
                                    size_t len);
int dpf_amd_dcf_generate_keys(dpf_amd_dcf* dcf, uint64_t alpha_lo,
                              uint64_t alpha_hi, const uint8_t* beta,
                              size_t beta_len, const uint64_t* seeds,
                              uint8_t** key0, size_t* key0_len,
                              uint8_t** key1, size_t* key1_len);
int dpf_amd_dcf_batch_evaluate(const dpf_amd_dcf* dcf,
                               const uint8_t* const* keys,
                               const size_t* key_lengths, int64_t num_keys,
                               const uint64_t* points, int64_t num_points,
                               const uint8_t* value_type,
                               size_t value_type_len, void* out);

/* Dense PIR database: DenseDpfPirDatabase::Builder (pir/dense_dpf_pir_database.h
 * :41-62) with the records resident in HBM. */
int dpf_amd_pir_db_create(dpf_amd_pir_db** out);
int dpf_amd_pir_db_insert(dpf_amd_pir_db* db, const uint8_t* record,
                          size_t len);
/* Bulk insert of num_records records of equal size. */
int dpf_amd_pir_db_insert_fixed(dpf_amd_pir_db* db, const uint8_t* records,
                                int64_t num_records, int64_t record_size);
/* Bulk insert of num_records records of any sizes, concatenated in `data`
 * (record i is sizes[i] bytes): Builder::Insert for each, in order. */
int dpf_amd_pir_db_insert_packed(dpf_amd_pir_db* db, const uint8_t* data,
                                 const int64_t* sizes, int64_t num_records);
/* Bulk insert of num_records records of record_size bytes that already live
 * in device memory on `device` (consecutive); Build copies them device to
 * device, never through the host. Must be the only insert of the database. */
int dpf_amd_pir_db_insert_fixed_device(dpf_amd_pir_db* db, const void* records,
                                       int device, int64_t num_records,
                                       int64_t record_size);
int dpf_amd_pir_db_build(dpf_amd_pir_db* db);
void dpf_amd_pir_db_destroy(dpf_amd_pir_db* db);
int64_t dpf_amd_pir_db_size(const dpf_amd_pir_db* db);
int64_t dpf_amd_pir_db_max_value_size(const dpf_amd_pir_db* db);
/* Shards the records over devices before dpf_amd_pir_db_build: contiguous
 * row ranges aligned to 128-record selection blocks, one per entry of
 * `devices` (entries may repeat). HandleRequest / InnerProductWith then scan
 * every shard on its device and combine the Q x record partials on the first
 * shard's device (peer copies over xGMI + one XOR fold). No call, or
 * num_devices = 0: one shard on the current device. */
int dpf_amd_pir_db_set_devices(dpf_amd_pir_db* db, const int* devices,
                               int num_devices);
int dpf_amd_pir_db_num_shards(const dpf_amd_pir_db* db);
/* Shard `shard` of a built database: device, rows [row_begin, row_end),
 * device pointer of its records (record stride: dpf_amd_pir_db_device_records).
 * Any output pointer may be NULL. */
int dpf_amd_pir_db_shard(const dpf_amd_pir_db* db, int shard, int* device,
                         int64_t* row_begin, int64_t* row_end,
                         const void** records);
/* Device pointer / stride of the resident records of shard 0 (bench). */
const void* dpf_amd_pir_db_device_records(const dpf_amd_pir_db* db,
                                          int64_t* record_stride);
/* PirDatabaseInterface::InnerProductWith (pir/pir_database_interface.h:65-66):
 * selections are host arrays of num_queries * selection_blocks 128-bit blocks;
 * out receives num_queries * max_value_size bytes. */
int dpf_amd_pir_db_inner_product(const dpf_amd_pir_db* db,
                                 const uint64_t* selections,
                                 int64_t selection_blocks, int num_queries,
                                 uint8_t* out);

/* DenseDpfPirServer::CreatePlain (pir/dense_dpf_pir_server.h:84-86) from a
 * serialized PirConfig; takes ownership of `db`. */
int dpf_amd_pir_server_create_plain(const uint8_t* config, size_t config_len,
                                    dpf_amd_pir_db* db,
                                    dpf_amd_pir_server** out);
void dpf_amd_pir_server_destroy(dpf_amd_pir_server* server);
/* Leader / Helper roles (pir/dense_dpf_pir_server.h:65-82,
 * pir/dpf_pir_server.cc:55-193). The reference's callbacks
 * ForwardHelperRequestFn / DecryptHelperRequestFn (pir/dpf_pir_server.h:92-
 * 109) become C function pointers that talk back through a call handle:
 *   forward(helper_request, len, call, user): send the serialized PirRequest
 *     to the Helper; while waiting for it call
 *     dpf_amd_pir_call_while_waiting(call) (the Leader computes its own share
 *     there), then hand the Helper's serialized PirResponse to
 *     dpf_amd_pir_call_set_response(call, ...). Return 0, or a status code.
 *   decrypt(ciphertext, len, context_info, info_len, call, user): decrypt the
 *     EncryptedHelperRequest (Tink HybridDecrypt in the reference) and hand
 *     the plaintext HelperRequest to dpf_amd_pir_call_set_response. */
typedef struct dpf_amd_pir_call dpf_amd_pir_call;
typedef int (*dpf_amd_pir_forward_fn)(const uint8_t* helper_request, size_t len,
                                      dpf_amd_pir_call* call, void* user);
typedef int (*dpf_amd_pir_decrypt_fn)(const uint8_t* ciphertext, size_t len,
                                      const uint8_t* context_info,
                                      size_t info_len, dpf_amd_pir_call* call,
                                      void* user);
int dpf_amd_pir_call_while_waiting(dpf_amd_pir_call* call);
int dpf_amd_pir_call_set_response(dpf_amd_pir_call* call, const uint8_t* data,
                                  size_t len);
int dpf_amd_pir_server_create_leader(const uint8_t* config, size_t config_len,
                                     dpf_amd_pir_db* db,
                                     dpf_amd_pir_forward_fn forward, void* user,
                                     dpf_amd_pir_server** out);
int dpf_amd_pir_server_create_helper(const uint8_t* config, size_t config_len,
                                     dpf_amd_pir_db* db,
                                     dpf_amd_pir_decrypt_fn decrypt, void* user,
                                     dpf_amd_pir_server** out);
/* DpfPirServer::HandleRequest (pir/dpf_pir_server.h:123-124): serialized
 * PirRequest in, serialized PirResponse out. */
int dpf_amd_pir_server_handle_request(const dpf_amd_pir_server* server,
                                      const uint8_t* request,
                                      size_t request_len, uint8_t** response,
                                      size_t* response_len);

/* ---- Cuckoo-hashed sparse (keyword) PIR ------------------------------------
 * The reference's CuckooHashingSparseDpfPirServer
 * (pir/cuckoo_hashing_sparse_dpf_pir_server.h:37-125) over a
 * CuckooHashedDpfPirDatabase (pir/cuckoo_hashed_dpf_pir_database.h:37-110):
 * keys are cuckoo-placed into num_buckets buckets on the host, the key and
 * value tables live in HBM, and one request is one DPF expansion per key plus
 * two HBM scans. Servers share the dpf_amd_pir_server handle (HandleRequest,
 * destroy) with the dense server. */
typedef struct dpf_amd_cuckoo_db dpf_amd_cuckoo_db;

/* SHA256HashFunction(seed)(input, upper_bound)
 * (pir/hashing/sha256_hash_family.cc:59-86). */
int dpf_amd_sha256_hash(const uint8_t* seed, size_t seed_len,
                        const uint8_t* input, size_t input_len, int upper_bound,
                        int* out);
/* CreateHashFunctions(CreateHashFamilyFromConfig(config), n)[i](input, ub)
 * for i < n into out[0..n) (pir/hashing/hash_family.cc:27-39,
 * hash_family_config.cc:27-45); `hash_family_config` is a serialized
 * HashFamilyConfig. */
int dpf_amd_hash_family_evaluate(const uint8_t* hash_family_config,
                                 size_t config_len, int num_hash_functions,
                                 const uint8_t* input, size_t input_len,
                                 int upper_bound, int* out);
/* CuckooHashingSparseDpfPirServer::GenerateParams (.cc:46-65): serialized
 * PirConfig in, serialized CuckooHashingParams out (free with dpf_amd_free). */
int dpf_amd_cuckoo_generate_params(const uint8_t* config, size_t config_len,
                                   uint8_t** params, size_t* params_len);
/* CuckooHashedDpfPirDatabase::Builder (SetParams / Insert / Build). */
int dpf_amd_cuckoo_db_create(const uint8_t* params, size_t params_len,
                             dpf_amd_cuckoo_db** out);
int dpf_amd_cuckoo_db_insert(dpf_amd_cuckoo_db* db, const uint8_t* key,
                             size_t key_len, const uint8_t* value,
                             size_t value_len);
/* Host-only cuckoo placement of the inserted keys (the first half of
 * Build(), cuckoo_hashed_dpf_pir_database.cc:100-131): bucket_key_lengths[b]
 * = length of the key in bucket b, or -1 when empty; place_keys writes the
 * placed keys back to back in bucket order. */
int dpf_amd_cuckoo_db_place(const dpf_amd_cuckoo_db* db,
                            int64_t* bucket_key_lengths, int64_t num_buckets);
int dpf_amd_cuckoo_db_place_keys(const dpf_amd_cuckoo_db* db, uint8_t* keys,
                                 size_t keys_len);
int dpf_amd_cuckoo_db_build(dpf_amd_cuckoo_db* db);
void dpf_amd_cuckoo_db_destroy(dpf_amd_cuckoo_db* db);
int64_t dpf_amd_cuckoo_db_size(const dpf_amd_cuckoo_db* db);
int64_t dpf_amd_cuckoo_db_num_selection_bits(const dpf_amd_cuckoo_db* db);
/* CuckooHashingSparseDpfPirServer::{CreatePlain, CreateLeader, CreateHelper}
 * (.cc:67-128) from serialized CuckooHashingParams; take ownership of `db`
 * (built here if needed). */
int dpf_amd_cuckoo_server_create_plain(const uint8_t* params, size_t params_len,
                                       dpf_amd_cuckoo_db* db,
                                       dpf_amd_pir_server** out);
int dpf_amd_cuckoo_server_create_leader(const uint8_t* params,
                                        size_t params_len, dpf_amd_cuckoo_db* db,
                                        dpf_amd_pir_forward_fn forward,
                                        void* user, dpf_amd_pir_server** out);
int dpf_amd_cuckoo_server_create_helper(const uint8_t* params,
                                        size_t params_len, dpf_amd_cuckoo_db* db,
                                        dpf_amd_pir_decrypt_fn decrypt,
                                        void* user, dpf_amd_pir_server** out);
/* PirServer::GetPublicParams (pir/pir_server.h): serialized
 * PirServerPublicParams. */
int dpf_amd_pir_server_public_params(const dpf_amd_pir_server* server,
                                     uint8_t** params, size_t* params_len);

#ifdef __cplusplus
}
#endif
#endif
