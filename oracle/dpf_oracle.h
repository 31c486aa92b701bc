/*
 * dpf_oracle.h — CPU ORACLE (TEST INFRASTRUCTURE ONLY).
 *
 * A plain-C restatement of the reference's CPU semantics for the DPF tree
 * expansion + dense-PIR scan hot path (d346uvcdd/distributed_point_functions,
 * mounted read-only at /root/reference).  It exists to CHECK the HIP product
 * path and to time the reference-faithful CPU algorithm (bench.py's
 * `cpu_baseline`).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it; the product (distributed_point_functions_amd/)
 * never links, loads or calls it.
 *
 * Parity pinning:
 *   - AES-MMO known-answer vectors of dpf/aes_128_fixed_key_hash_test.cc:120-141
 *   - IntModN sampling KAT of dpf/int_mod_n_test.cc:162-193
 *   - Tuple FromBytes KATs of dpf/internal/value_type_helpers_test.cc:230-255
 *   - OpenSSL libcrypto AES-128-ECB cross-check (same AES the reference links)
 *   - the reference's share-sum property tests (distributed_point_function_test.cc)
 * The reference itself cannot be built here (Bazel + Abseil + Highway +
 * BoringSSL + protobuf runtime absent, no network), so there is no oracle/_ref.
 *
 * Conventions: every 128-bit quantity crosses this ABI as two uint64 words
 * {lo, hi} (the little-endian memory layout of absl::uint128 / unsigned
 * __int128 on x86-64).  Status codes are absl::StatusCode numbers.
 */
#ifndef DPF_ORACLE_H_
#define DPF_ORACLE_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  OR_OK = 0,
  OR_INVALID_ARGUMENT = 3,
  OR_RESOURCE_EXHAUSTED = 8,
  OR_FAILED_PRECONDITION = 9,
  OR_UNIMPLEMENTED = 12,
  OR_INTERNAL = 13,
};

/* ValueType node, pre-order serialised (proto field numbers as kinds):
 *   kind 1 = Integer{bitsize}, 2 = Tuple{n_children nodes follow},
 *   3 = IntModN{base bitsize, modulus}, 4 = XorWrapper{bitsize}. */
typedef struct {
  int32_t kind;
  int32_t bits;
  int32_t n_children;
  int32_t reserved;
  uint64_t mod_lo, mod_hi;
} or_vt_node;

const char* or_last_error(void);

/* a1: Aes128FixedKeyHash::Evaluate (aes_128_fixed_key_hash.cc:57-98). */
int or_aes_mmo(uint64_t key_lo, uint64_t key_hi, const uint64_t* in,
               uint64_t* out, int64_t n);
/* Raw AES-128 single block encryption (for KAT / OpenSSL cross-checks). */
void or_aes128_encrypt_block(const uint8_t key[16], const uint8_t in[16],
                             uint8_t out[16]);
int or_have_aesni(void);
void or_force_portable_aes(int on);

/* value_type_helpers.cc:71-141 */
int or_bits_needed(const or_vt_node* vt, double security_parameter,
                   int* bits_out);
/* int_mod_n.cc:71-84 */
int or_intmodn_num_bytes_required(int num_samples, int base_bits,
                                  uint64_t mod_lo, uint64_t mod_hi,
                                  double security_parameter, int* out);
/* Number of flattened scalars, elements per block, directly-convertible. */
int or_vt_num_scalars(const or_vt_node* vt);
int or_vt_elements_per_block(const or_vt_node* vt);
int or_vt_directly_convertible(const or_vt_node* vt);
/* ConvertBytesToArrayOf<T> (vth:586-606): out = epb * num_scalars words(2). */
int or_convert_bytes(const or_vt_node* vt, const uint8_t* bytes, int64_t len,
                     uint64_t* out);
/* IntModNImpl::UnsafeSampleFromBytes (int_mod_n.h:159-182). */
void or_intmodn_sample(const uint8_t* bytes, int base_bytes, uint64_t mod_lo,
                       uint64_t mod_hi, int num_samples, uint64_t* out);

/* ---------------------------------------------------------------------- */
/* DPF object: DistributedPointFunction::CreateIncremental (cc:589-640)    */
typedef struct or_dpf or_dpf;

/* `vt_nodes` holds the value types of all levels back to back;
 * `vt_node_counts[i]` nodes belong to level i. */
int or_dpf_create(int num_levels, const int32_t* log_domain_sizes,
                  const double* security_parameters, const or_vt_node* vt_nodes,
                  const int32_t* vt_node_counts, or_dpf** out);
void or_dpf_free(or_dpf* dpf);
int or_dpf_tree_levels_needed(const or_dpf* dpf);
int or_dpf_hierarchy_to_tree(const or_dpf* dpf, int h);
int or_dpf_blocks_needed(const or_dpf* dpf, int h);
int or_dpf_num_scalars(const or_dpf* dpf, int h);
int or_dpf_elements_per_block(const or_dpf* dpf, int h);
double or_dpf_security_parameter(const or_dpf* dpf, int h);

/* Flat DpfKey: correction words SoA for tree levels 1..L-1, and per-hierarchy
 * value corrections vc[h] (epb_h * ns_h 128-bit words), which is where the
 * proto keeps them: correction_words[h2t[h]].value_correction, or
 * last_level_value_correction for the last level (h:815-827). */
typedef struct {
  uint64_t seed[2];
  int32_t party;
  int32_t num_cw;
  uint64_t* cw_seed;   /* num_cw * 2 */
  uint8_t* cw_ccl;     /* num_cw */
  uint8_t* cw_ccr;     /* num_cw */
  int32_t num_levels;
  int32_t* vc_count;   /* num_levels: number of 128-bit words */
  uint64_t* vc;        /* concatenated, 2 words each */
} or_key;

/* GenerateKeysIncremental (cc:642-710) with injected root seeds replacing
 * RAND_bytes (cc:680-681).  beta: concatenated flattened scalars per level. */
int or_generate_keys(const or_dpf* dpf, uint64_t alpha_lo, uint64_t alpha_hi,
                     const uint64_t* beta, const uint64_t seeds[4],
                     or_key** key0, or_key** key1);
void or_key_free(or_key* key);
or_key* or_key_alloc(int num_cw, int num_levels, const int32_t* vc_count);

/* EvaluationContext (proto:156-171) state. */
typedef struct or_ctx or_ctx;
int or_ctx_create(const or_dpf* dpf, const or_key* key, or_ctx** out);
void or_ctx_free(or_ctx* ctx);
int or_ctx_previous_hierarchy_level(const or_ctx* ctx);
int or_ctx_partial_evaluations_level(const or_ctx* ctx);
int64_t or_ctx_num_partial_evaluations(const or_ctx* ctx);
/* prefix, seed: 2 words each; control bit 1 byte. */
void or_ctx_partial_evaluations(const or_ctx* ctx, uint64_t* prefixes,
                                uint64_t* seeds, uint8_t* control_bits);

/* EvaluateUntil<T> (h:695-891).  Output: out_count elements, each
 * num_scalars 128-bit words (element-major).  `out` may be NULL to query
 * *out_count. */
int or_evaluate_until(const or_dpf* dpf, int hierarchy_level,
                      const uint64_t* prefixes, int64_t num_prefixes,
                      or_ctx* ctx, uint64_t* out, int64_t out_capacity,
                      int64_t* out_count);

/* EvaluateAt<T>(key, level, points) (h:913-1070, ctx == nullptr). */
int or_evaluate_at(const or_dpf* dpf, const or_key* key, int hierarchy_level,
                   const uint64_t* points, int64_t num_points, uint64_t* out);

/* EvaluateAt<T>(level, points, ctx) (h:356-378, 1000-1011): starts from the
 * partial evaluations in `ctx` and rewrites them at `hierarchy_level`. */
int or_evaluate_at_ctx(const or_dpf* dpf, int hierarchy_level, const uint64_t* points,
                       int64_t num_points, or_ctx* ctx, uint64_t* out);

/* dpf_internal::EvaluateSeeds (evaluate_prg_hwy.cc:552-658): generic keys. */
int or_evaluate_seeds(int64_t num_seeds, int num_levels,
                      int64_t num_correction_words, const uint64_t* seeds_in,
                      const uint8_t* control_bits_in, const uint64_t* paths,
                      int paths_rightshift, const uint64_t* correction_seeds,
                      const uint8_t* ccl, const uint8_t* ccr,
                      uint64_t key_left_lo, uint64_t key_left_hi,
                      uint64_t key_right_lo, uint64_t key_right_hi,
                      uint64_t* seeds_out, uint8_t* control_bits_out);

/* Bounded full-domain slice for the CPU baseline: evaluates the last
 * hierarchy level of `key` on the aligned leaf-block range
 * [first_block, first_block + 2^log_blocks) of the tree (path walk to the
 * subtree root, then ExpandSeeds + HashExpandedSeeds + correction exactly as
 * EvaluateUntil does).  out: 2^log_blocks * cepb elements. */
int or_expand_subtree(const or_dpf* dpf, const or_key* key, uint64_t first_lo,
                      uint64_t first_hi, int log_blocks, uint64_t* out);

/* pir_internal::InnerProductNoHwy + InnerProduct validation
 * (inner_product_hwy.cc:270-334).  values: concatenated record bytes with
 * offsets/sizes; selections: num_queries * num_blocks 128-bit words;
 * out: num_queries * max_value_size bytes. */
int or_inner_product(int64_t num_values, const uint8_t* data,
                     const int64_t* offsets, const int64_t* sizes,
                     int num_queries, int64_t num_blocks,
                     const uint64_t* selections, int64_t max_value_size,
                     uint8_t* out);

/* Aes128CtrSeededPrng::GetRandomBytes from a fresh PRNG with zero nonce
 * (aes_128_ctr_seeded_prng.cc:60-101). */
void or_aes_ctr_prng(const uint8_t seed[16], int64_t length, uint8_t* out);

#ifdef __cplusplus
}
#endif
#endif
