/*
 * dpf_oracle.c — CPU ORACLE (TEST INFRASTRUCTURE ONLY; see dpf_oracle.h).
 *
 * Plain C restatement of the reference CPU path.  Every function cites the
 * reference file:line it follows ("cc" = dpf/distributed_point_function.cc,
 * "h" = dpf/distributed_point_function.h, "vth" =
 * dpf/internal/value_type_helpers.h).  Loop structure follows the reference
 * (64-block AES batches in ExpandSeeds, per-leaf correction loop) so that the
 * bench's cpu_baseline times the reference's algorithm.
 */
#include "dpf_oracle.h"

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

typedef unsigned __int128 u128;

#define U128(lo, hi) (((u128)(uint64_t)(hi) << 64) | (u128)(uint64_t)(lo))
#define LO64(x) ((uint64_t)(x))
#define HI64(x) ((uint64_t)((x) >> 64))

static __thread char g_err[1024];

const char* or_last_error(void) { return g_err; }

static int set_err(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

static void u128_to_dec(u128 v, char* buf) {
  char tmp[64];
  int n = 0;
  if (v == 0) tmp[n++] = '0';
  while (v) {
    tmp[n++] = (char)('0' + (int)(v % 10));
    v /= 10;
  }
  for (int i = 0; i < n; ++i) buf[i] = tmp[n - 1 - i];
  buf[n] = 0;
}

static inline u128 load_u128(const uint64_t* p) { return U128(p[0], p[1]); }
static inline void store_u128(uint64_t* p, u128 v) {
  p[0] = LO64(v);
  p[1] = HI64(v);
}

/* ======================================================================== */
/* AES-128 (FIPS-197).  The reference uses BoringSSL EVP AES-128-ECB.       */
/* ======================================================================== */

static const uint8_t kSbox[256] = {
    0x63, 0x7c, 0x77, 0x7b, 0xf2, 0x6b, 0x6f, 0xc5, 0x30, 0x01, 0x67, 0x2b,
    0xfe, 0xd7, 0xab, 0x76, 0xca, 0x82, 0xc9, 0x7d, 0xfa, 0x59, 0x47, 0xf0,
    0xad, 0xd4, 0xa2, 0xaf, 0x9c, 0xa4, 0x72, 0xc0, 0xb7, 0xfd, 0x93, 0x26,
    0x36, 0x3f, 0xf7, 0xcc, 0x34, 0xa5, 0xe5, 0xf1, 0x71, 0xd8, 0x31, 0x15,
    0x04, 0xc7, 0x23, 0xc3, 0x18, 0x96, 0x05, 0x9a, 0x07, 0x12, 0x80, 0xe2,
    0xeb, 0x27, 0xb2, 0x75, 0x09, 0x83, 0x2c, 0x1a, 0x1b, 0x6e, 0x5a, 0xa0,
    0x52, 0x3b, 0xd6, 0xb3, 0x29, 0xe3, 0x2f, 0x84, 0x53, 0xd1, 0x00, 0xed,
    0x20, 0xfc, 0xb1, 0x5b, 0x6a, 0xcb, 0xbe, 0x39, 0x4a, 0x4c, 0x58, 0xcf,
    0xd0, 0xef, 0xaa, 0xfb, 0x43, 0x4d, 0x33, 0x85, 0x45, 0xf9, 0x02, 0x7f,
    0x50, 0x3c, 0x9f, 0xa8, 0x51, 0xa3, 0x40, 0x8f, 0x92, 0x9d, 0x38, 0xf5,
    0xbc, 0xb6, 0xda, 0x21, 0x10, 0xff, 0xf3, 0xd2, 0xcd, 0x0c, 0x13, 0xec,
    0x5f, 0x97, 0x44, 0x17, 0xc4, 0xa7, 0x7e, 0x3d, 0x64, 0x5d, 0x19, 0x73,
    0x60, 0x81, 0x4f, 0xdc, 0x22, 0x2a, 0x90, 0x88, 0x46, 0xee, 0xb8, 0x14,
    0xde, 0x5e, 0x0b, 0xdb, 0xe0, 0x32, 0x3a, 0x0a, 0x49, 0x06, 0x24, 0x5c,
    0xc2, 0xd3, 0xac, 0x62, 0x91, 0x95, 0xe4, 0x79, 0xe7, 0xc8, 0x37, 0x6d,
    0x8d, 0xd5, 0x4e, 0xa9, 0x6c, 0x56, 0xf4, 0xea, 0x65, 0x7a, 0xae, 0x08,
    0xba, 0x78, 0x25, 0x2e, 0x1c, 0xa6, 0xb4, 0xc6, 0xe8, 0xdd, 0x74, 0x1f,
    0x4b, 0xbd, 0x8b, 0x8a, 0x70, 0x3e, 0xb5, 0x66, 0x48, 0x03, 0xf6, 0x0e,
    0x61, 0x35, 0x57, 0xb9, 0x86, 0xc1, 0x1d, 0x9e, 0xe1, 0xf8, 0x98, 0x11,
    0x69, 0xd9, 0x8e, 0x94, 0x9b, 0x1e, 0x87, 0xe9, 0xce, 0x55, 0x28, 0xdf,
    0x8c, 0xa1, 0x89, 0x0d, 0xbf, 0xe6, 0x42, 0x68, 0x41, 0x99, 0x2d, 0x0f,
    0xb0, 0x54, 0xbb, 0x16};

static void aes128_expand_key(const uint8_t key[16], uint8_t rk[176]) {
  static const uint8_t rcon[10] = {0x01, 0x02, 0x04, 0x08, 0x10,
                                   0x20, 0x40, 0x80, 0x1b, 0x36};
  memcpy(rk, key, 16);
  for (int i = 4; i < 44; ++i) {
    uint8_t t[4];
    memcpy(t, rk + 4 * (i - 1), 4);
    if (i % 4 == 0) {
      uint8_t u = t[0];
      t[0] = (uint8_t)(kSbox[t[1]] ^ rcon[i / 4 - 1]);
      t[1] = kSbox[t[2]];
      t[2] = kSbox[t[3]];
      t[3] = kSbox[u];
    }
    for (int j = 0; j < 4; ++j) rk[4 * i + j] = rk[4 * (i - 4) + j] ^ t[j];
  }
}

static inline uint8_t xtime(uint8_t x) {
  return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1b : 0));
}

static void aes128_encrypt_portable(const uint8_t rk[176], const uint8_t in[16],
                                    uint8_t out[16]) {
  uint8_t s[16];
  for (int i = 0; i < 16; ++i) s[i] = in[i] ^ rk[i];
  for (int round = 1; round <= 10; ++round) {
    uint8_t t[16];
    /* SubBytes + ShiftRows: state byte (r, c) = s[r + 4c]. */
    for (int c = 0; c < 4; ++c)
      for (int r = 0; r < 4; ++r) t[r + 4 * c] = kSbox[s[r + 4 * ((c + r) & 3)]];
    if (round != 10) {
      for (int c = 0; c < 4; ++c) {
        uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2],
                a3 = t[4 * c + 3];
        uint8_t all = a0 ^ a1 ^ a2 ^ a3;
        t[4 * c] = a0 ^ all ^ xtime(a0 ^ a1);
        t[4 * c + 1] = a1 ^ all ^ xtime(a1 ^ a2);
        t[4 * c + 2] = a2 ^ all ^ xtime(a2 ^ a3);
        t[4 * c + 3] = a3 ^ all ^ xtime(a3 ^ a0);
      }
    }
    for (int i = 0; i < 16; ++i) s[i] = t[i] ^ rk[16 * round + i];
  }
  memcpy(out, s, 16);
}

static int g_force_portable = 0;
void or_force_portable_aes(int on) { g_force_portable = on; }

int or_have_aesni(void) {
#if defined(__x86_64__)
  return __builtin_cpu_supports("aes") && !g_force_portable;
#else
  return 0;
#endif
}

#if defined(__x86_64__)
__attribute__((target("aes,sse4.1"))) static void aesni_encrypt_blocks(
    const uint8_t rk[176], const uint8_t* in, uint8_t* out, int64_t n) {
  __m128i k[11];
  for (int i = 0; i < 11; ++i) k[i] = _mm_loadu_si128((const __m128i*)(rk + 16 * i));
  int64_t i = 0;
  for (; i + 8 <= n; i += 8) {
    __m128i b[8];
    for (int j = 0; j < 8; ++j)
      b[j] = _mm_xor_si128(_mm_loadu_si128((const __m128i*)(in + 16 * (i + j))), k[0]);
    for (int r = 1; r < 10; ++r)
      for (int j = 0; j < 8; ++j) b[j] = _mm_aesenc_si128(b[j], k[r]);
    for (int j = 0; j < 8; ++j)
      _mm_storeu_si128((__m128i*)(out + 16 * (i + j)), _mm_aesenclast_si128(b[j], k[10]));
  }
  for (; i < n; ++i) {
    __m128i b = _mm_xor_si128(_mm_loadu_si128((const __m128i*)(in + 16 * i)), k[0]);
    for (int r = 1; r < 10; ++r) b = _mm_aesenc_si128(b, k[r]);
    _mm_storeu_si128((__m128i*)(out + 16 * i), _mm_aesenclast_si128(b, k[10]));
  }
}
#endif

static void aes128_encrypt_blocks(const uint8_t rk[176], const uint8_t* in,
                                  uint8_t* out, int64_t n) {
#if defined(__x86_64__)
  if (or_have_aesni()) {
    aesni_encrypt_blocks(rk, in, out, n);
    return;
  }
#endif
  for (int64_t i = 0; i < n; ++i) aes128_encrypt_portable(rk, in + 16 * i, out + 16 * i);
}

void or_aes128_encrypt_block(const uint8_t key[16], const uint8_t in[16],
                             uint8_t out[16]) {
  uint8_t rk[176];
  aes128_expand_key(key, rk);
  aes128_encrypt_blocks(rk, in, out, 1);
}

/* Aes128FixedKeyHash (aes_128_fixed_key_hash.cc:37-98): key bytes are the
 * little-endian bytes of the uint128 key (.cc:49-50). */
typedef struct {
  uint8_t rk[176];
} or_prg;

static void prg_init(or_prg* prg, u128 key) {
  uint8_t kb[16];
  memcpy(kb, &key, 16); /* little-endian host == reinterpret_cast */
  aes128_expand_key(kb, prg->rk);
}

enum { kBatchSize = 64 }; /* aes_128_fixed_key_hash.h:70 */

/* out[i] = AES(sigma(in[i])) ^ sigma(in[i]); sigma(x) = (hi^lo, hi)
 * (aes_128_fixed_key_hash.cc:66-96).  In-place safe. */
static void prg_evaluate(const or_prg* prg, const u128* in, u128* out,
                         int64_t n) {
  u128 sigma_in[kBatchSize];
  for (int64_t start = 0; start < n; start += kBatchSize) {
    int64_t bs = n - start < kBatchSize ? n - start : kBatchSize;
    for (int64_t i = 0; i < bs; ++i) {
      u128 x = in[start + i];
      sigma_in[i] = U128(HI64(x), HI64(x) ^ LO64(x));
    }
    aes128_encrypt_blocks(prg->rk, (const uint8_t*)sigma_in,
                          (uint8_t*)(out + start), bs);
    for (int64_t i = 0; i < bs; ++i) out[start + i] ^= sigma_in[i];
  }
}

int or_aes_mmo(uint64_t key_lo, uint64_t key_hi, const uint64_t* in,
               uint64_t* out, int64_t n) {
  or_prg prg;
  prg_init(&prg, U128(key_lo, key_hi));
  u128* buf = (u128*)malloc(sizeof(u128) * (size_t)(n > 0 ? n : 1));
  if (!buf) return set_err(OR_RESOURCE_EXHAUSTED, "Memory allocation error");
  for (int64_t i = 0; i < n; ++i) buf[i] = load_u128(in + 2 * i);
  prg_evaluate(&prg, buf, buf, n);
  for (int64_t i = 0; i < n; ++i) store_u128(out + 2 * i, buf[i]);
  free(buf);
  return OR_OK;
}

/* PRG keys (cc:55-60). */
static const u128 kPrgKeyLeft =
    U128(0x935f08d0a5b6a2fdULL, 0x5be037ccf6a03de5ULL);
static const u128 kPrgKeyRight =
    U128(0xe2ea1fe0f66f4d0bULL, 0xef94b6aedebb026cULL);
static const u128 kPrgKeyValue =
    U128(0x46a31101b21d1c98ULL, 0x05a5d1588c5423e3ULL);

/* ======================================================================== */
/* Value types (vth, value_type_helpers.cc, int_mod_n.{h,cc})                */
/* ======================================================================== */

typedef struct {
  int kind; /* 1 integer, 3 int_mod_n, 4 xor_wrapper */
  int bits;
  u128 modulus;
} scalar_t;

#define MAX_SCALARS 64
#define MAX_VT_NODES 128

typedef struct {
  int num_nodes;
  or_vt_node nodes[MAX_VT_NODES];
  int num_scalars;
  scalar_t scalars[MAX_SCALARS];
  int direct;     /* can_be_converted_directly */
  int total_bits; /* TotalBitSize for direct types */
  int epb;        /* ElementsPerBlock */
  int esz;        /* element size in bytes (direct) */
} vtype_t;

/* Returns number of nodes consumed by the subtree at `vt`, or -1. */
static int vt_subtree_size(const or_vt_node* vt, int avail) {
  if (avail <= 0) return -1;
  if (vt[0].kind != 2) return 1;
  int used = 1;
  for (int i = 0; i < vt[0].n_children; ++i) {
    int s = vt_subtree_size(vt + used, avail - used);
    if (s < 0) return -1;
    used += s;
  }
  return used;
}

static int vt_flatten(const or_vt_node* vt, vtype_t* out, int* pos) {
  const or_vt_node* n = vt + *pos;
  (*pos)++;
  if (n->kind == 2) {
    for (int i = 0; i < n->n_children; ++i)
      if (vt_flatten(vt, out, pos) != OR_OK) return OR_INVALID_ARGUMENT;
    return OR_OK;
  }
  if (out->num_scalars >= MAX_SCALARS)
    return set_err(OR_UNIMPLEMENTED, "too many tuple elements");
  scalar_t* s = &out->scalars[out->num_scalars++];
  s->kind = n->kind;
  s->bits = n->bits;
  s->modulus = U128(n->mod_lo, n->mod_hi);
  if (n->kind != 1 && n->kind != 3 && n->kind != 4)
    return set_err(OR_INVALID_ARGUMENT, "Unsupported ValueType kind %d", n->kind);
  return OR_OK;
}

static int vt_build(const or_vt_node* nodes, int count, vtype_t* vt) {
  memset(vt, 0, sizeof(*vt));
  if (count <= 0 || count > MAX_VT_NODES)
    return set_err(OR_INVALID_ARGUMENT, "bad value type");
  int sz = vt_subtree_size(nodes, count);
  if (sz != count) return set_err(OR_INVALID_ARGUMENT, "malformed value type");
  memcpy(vt->nodes, nodes, sizeof(or_vt_node) * (size_t)count);
  vt->num_nodes = count;
  int pos = 0;
  int st = vt_flatten(nodes, vt, &pos);
  if (st != OR_OK) return st;
  vt->direct = 1;
  vt->total_bits = 0;
  for (int i = 0; i < vt->num_scalars; ++i) {
    if (vt->scalars[i].kind == 3) vt->direct = 0;
    vt->total_bits += vt->scalars[i].bits;
  }
  /* ElementsPerBlock (vth:525-537). */
  if (vt->direct && vt->total_bits <= 128)
    vt->epb = 128 / vt->total_bits;
  else
    vt->epb = 1;
  vt->esz = (vt->total_bits + 7) / 8;
  return OR_OK;
}

int or_vt_num_scalars(const or_vt_node* vt) {
  vtype_t t;
  int c = vt_subtree_size(vt, MAX_VT_NODES);
  if (c < 0 || vt_build(vt, c, &t) != OR_OK) return -1;
  return t.num_scalars;
}
int or_vt_elements_per_block(const or_vt_node* vt) {
  vtype_t t;
  int c = vt_subtree_size(vt, MAX_VT_NODES);
  if (c < 0 || vt_build(vt, c, &t) != OR_OK) return -1;
  return t.epb;
}
int or_vt_directly_convertible(const or_vt_node* vt) {
  vtype_t t;
  int c = vt_subtree_size(vt, MAX_VT_NODES);
  if (c < 0 || vt_build(vt, c, &t) != OR_OK) return -1;
  return t.direct;
}

/* absl::uint128 -> double (absl int128.h): lo + ldexp(hi, 64). */
static double u128_to_double(u128 v) {
  return (double)LO64(v) + ldexp((double)HI64(v), 64);
}

/* IntModNBase::GetSecurityLevel (int_mod_n.cc:29-34). */
static double intmodn_security_level(int num_samples, u128 modulus) {
  return 128 + 3 -
         (log2(u128_to_double(modulus)) + log2((double)num_samples) +
          log2((double)(num_samples + 1)));
}

/* IntModNBase::CheckParameters + GetNumBytesRequired (int_mod_n.cc:36-84). */
static int intmodn_bytes_required(int num_samples, int base_bits, u128 modulus,
                                  double security_parameter, int* out) {
  if (num_samples <= 0)
    return set_err(OR_INVALID_ARGUMENT, "num_samples must be positive");
  if (base_bits <= 0)
    return set_err(OR_INVALID_ARGUMENT, "base_integer_bitsize must be positive");
  if (base_bits > 128)
    return set_err(OR_INVALID_ARGUMENT, "base_integer_bitsize must be at most 128");
  if (base_bits < 128 && ((u128)1 << base_bits) < modulus) {
    char m[64];
    u128_to_dec(modulus, m);
    return set_err(OR_INVALID_ARGUMENT,
                   "kModulus %s out of range for base_integer_bitsize = %d", m,
                   base_bits);
  }
  double sigma = intmodn_security_level(num_samples, modulus);
  if (security_parameter > sigma) {
    char m[64];
    u128_to_dec(modulus, m);
    return set_err(OR_INVALID_ARGUMENT,
                   "For num_samples = %d and kModulus = %s this approach can "
                   "only provide %f bits of statistical security. You can try "
                   "calling this function several times with smaller values "
                   "of num_samples.",
                   num_samples, m, sigma);
  }
  int base_bytes = (base_bits + 7) / 8;
  *out = 16 + base_bytes * (num_samples - 1);
  return OR_OK;
}

int or_intmodn_num_bytes_required(int num_samples, int base_bits,
                                  uint64_t mod_lo, uint64_t mod_hi,
                                  double security_parameter, int* out) {
  return intmodn_bytes_required(num_samples, base_bits, U128(mod_lo, mod_hi),
                                security_parameter, out);
}

/* ValueTypesAreEqual (value_type_helpers.cc:33-69) restricted to the
 * comparison BitsNeeded needs (IntModN elements). */
static int vt_nodes_equal_intmodn(const or_vt_node* a, const or_vt_node* b) {
  return a->kind == 3 && b->kind == 3 && a->bits == b->bits &&
         a->mod_lo == b->mod_lo && a->mod_hi == b->mod_hi;
}

/* BitsNeeded (value_type_helpers.cc:71-141), including the reference's
 * quirk of iterating elements(i) for i < num_other (lines 105-114). */
static int bits_needed_rec(const or_vt_node* vt, int avail,
                           double security_parameter, int* bits) {
  if (avail <= 0) return set_err(OR_INVALID_ARGUMENT, "malformed value type");
  switch (vt->kind) {
    case 1:
    case 4:
      *bits = vt->bits;
      return OR_OK;
    case 3: {
      int bytes;
      int st = intmodn_bytes_required(1, vt->bits, U128(vt->mod_lo, vt->mod_hi),
                                      security_parameter, &bytes);
      if (st != OR_OK) return st;
      *bits = 8 * bytes;
      return OR_OK;
    }
    case 2: {
      const or_vt_node* children[MAX_VT_NODES];
      int nchild = vt->n_children;
      int used = 1;
      for (int i = 0; i < nchild; ++i) {
        children[i] = vt + used;
        int s = vt_subtree_size(vt + used, avail - used);
        if (s < 0) return set_err(OR_INVALID_ARGUMENT, "malformed value type");
        used += s;
      }
      int num_ints_mod_n = 0, num_other = 0;
      const or_vt_node* int_mod_n = NULL;
      for (int i = 0; i < nchild; ++i) {
        if (children[i]->kind == 3) {
          if (!int_mod_n) {
            int_mod_n = children[i];
          } else if (!vt_nodes_equal_intmodn(children[i], int_mod_n)) {
            return set_err(OR_UNIMPLEMENTED,
                           "All elements of type IntModN in a tuple must be the same");
          }
          ++num_ints_mod_n;
        } else {
          ++num_other;
        }
      }
      int bitsize_other = 0, bitsize_ints_mod_n = 0;
      for (int i = 0; i < num_other; ++i) {
        double per_elem = security_parameter + log2((double)num_other);
        int el_bits;
        int st = bits_needed_rec(children[i], avail - (int)(children[i] - vt),
                                 per_elem, &el_bits);
        if (st != OR_OK) return st;
        bitsize_other += el_bits;
      }
      if (num_ints_mod_n > 0) {
        int bytes;
        int st = intmodn_bytes_required(
            num_ints_mod_n, int_mod_n->bits,
            U128(int_mod_n->mod_lo, int_mod_n->mod_hi), security_parameter,
            &bytes);
        if (st != OR_OK) return st;
        bitsize_ints_mod_n = bytes * 8;
      }
      *bits = bitsize_ints_mod_n + bitsize_other;
      return OR_OK;
    }
    default:
      return set_err(OR_INVALID_ARGUMENT, "BitsNeeded: Unsupported ValueType");
  }
}

int or_bits_needed(const or_vt_node* vt, double security_parameter,
                   int* bits_out) {
  int c = vt_subtree_size(vt, MAX_VT_NODES);
  if (c < 0) return set_err(OR_INVALID_ARGUMENT, "malformed value type");
  return bits_needed_rec(vt, c, security_parameter, bits_out);
}

/* --- scalar arithmetic (int_mod_n.h:121-250, xor_wrapper.h, tuple.h) --- */

static inline u128 mask_bits(int bits) {
  return bits >= 128 ? ~(u128)0 : (((u128)1 << bits) - 1);
}

static u128 s_add(const scalar_t* s, u128 a, u128 b) {
  switch (s->kind) {
    case 1:
      return (a + b) & mask_bits(s->bits);
    case 4:
      return a ^ b;
    default: { /* IntModN AddBaseInteger = SubtractBaseInteger(m - b) */
      u128 m = s->modulus, x = m - b;
      return a >= x ? a - x : m - x + a;
    }
  }
}

static u128 s_sub(const scalar_t* s, u128 a, u128 b) {
  switch (s->kind) {
    case 1:
      return (a - b) & mask_bits(s->bits);
    case 4:
      return a ^ b;
    default:
      return a >= b ? a - b : s->modulus - b + a;
  }
}

static u128 s_neg(const scalar_t* s, u128 a) {
  switch (s->kind) {
    case 1:
      return (0 - a) & mask_bits(s->bits);
    case 4:
      return a;
    default:
      return a == 0 ? 0 : s->modulus - a;
  }
}

static u128 le_bytes(const uint8_t* p, int n) {
  u128 v = 0;
  for (int i = n - 1; i >= 0; --i) v = (v << 8) | p[i];
  return v;
}

/* FromBytes<T> for one element (vth:543-555): `out` gets num_scalars words. */
static void element_from_bytes(const vtype_t* vt, const uint8_t* bytes,
                               int64_t len, u128* out) {
  if (vt->direct) {
    /* DirectlyFromBytes: consecutive little-endian byte slices. */
    int off = 0;
    for (int i = 0; i < vt->num_scalars; ++i) {
      int b = vt->scalars[i].bits / 8;
      out[i] = (off + b <= len) ? le_bytes(bytes + off, b) : 0;
      off += b;
    }
    return;
  }
  /* Sampling path (vth:230-251, 303-328, 447-460, 507-515): block = first 16
   * bytes; every scalar except the last flattened one updates the block. */
  u128 block = le_bytes(bytes, 16);
  int64_t pos = 16;
  for (int i = 0; i < vt->num_scalars; ++i) {
    const scalar_t* s = &vt->scalars[i];
    int update = (i + 1 < vt->num_scalars);
    int b = s->bits / 8;
    if (s->kind == 3) {
      u128 q = block / s->modulus, r = block % s->modulus;
      out[i] = r;
      if (update) {
        block = (b < 16) ? (q << (8 * b)) : 0;
        block |= (pos + b <= len) ? le_bytes(bytes + pos, b) : 0;
        pos += b;
      }
    } else {
      out[i] = block & mask_bits(s->bits);
      if (update) {
        if (b < 16)
          block &= ~mask_bits(s->bits);
        else
          block = 0;
        block |= (pos + b <= len) ? le_bytes(bytes + pos, b) : 0;
        pos += b;
      }
    }
  }
}

/* ConvertBytesToArrayOf<T> (vth:586-606): epb elements. */
static void convert_bytes_to_array(const vtype_t* vt, const uint8_t* bytes,
                                   int64_t len, u128* out) {
  if (vt->direct) {
    for (int e = 0; e < vt->epb; ++e)
      element_from_bytes(vt, bytes + (int64_t)e * vt->esz, vt->esz,
                         out + (int64_t)e * vt->num_scalars);
  } else {
    element_from_bytes(vt, bytes, len, out);
  }
}

int or_convert_bytes(const or_vt_node* nodes, const uint8_t* bytes, int64_t len,
                     uint64_t* out) {
  vtype_t vt;
  int c = vt_subtree_size(nodes, MAX_VT_NODES);
  if (c < 0) return set_err(OR_INVALID_ARGUMENT, "malformed value type");
  int st = vt_build(nodes, c, &vt);
  if (st != OR_OK) return st;
  u128 tmp[MAX_SCALARS * 16];
  convert_bytes_to_array(&vt, bytes, len, tmp);
  for (int i = 0; i < vt.epb * vt.num_scalars; ++i) store_u128(out + 2 * i, tmp[i]);
  return OR_OK;
}

void or_intmodn_sample(const uint8_t* bytes, int base_bytes, uint64_t mod_lo,
                       uint64_t mod_hi, int num_samples, uint64_t* out) {
  u128 m = U128(mod_lo, mod_hi);
  u128 r = le_bytes(bytes, 16);
  for (int i = 0; i < num_samples; ++i) {
    store_u128(out + 2 * i, r % m);
    if (i + 1 < num_samples) {
      r /= m;
      if (base_bytes < 16) r <<= 8 * base_bytes;
      r |= le_bytes(bytes + 16 + (int64_t)i * base_bytes, base_bytes);
    }
  }
}

/* ======================================================================== */
/* DPF object                                                                */
/* ======================================================================== */

struct or_dpf {
  int num_levels;
  int32_t log_domain[130];
  double security[130];
  vtype_t vt[130];
  int hierarchy_to_tree[130];
  int tree_to_hierarchy[130]; /* -1 if not an output level */
  int tree_levels_needed;
  int blocks_needed[130];
  or_prg prg_left, prg_right, prg_value;
};

int or_dpf_create(int num_levels, const int32_t* log_domain_sizes,
                  const double* security_parameters, const or_vt_node* vt_nodes,
                  const int32_t* vt_node_counts, or_dpf** out) {
  /* ProtoValidator::ValidateParameters (proto_validator.cc:160-203). */
  if (num_levels <= 0)
    return set_err(OR_INVALID_ARGUMENT, "`parameters` must not be empty");
  if (num_levels > 129)
    return set_err(OR_INVALID_ARGUMENT, "`log_domain_size` must be <= 128");
  or_dpf* d = (or_dpf*)calloc(1, sizeof(or_dpf));
  if (!d) return set_err(OR_RESOURCE_EXHAUSTED, "Memory allocation error");
  d->num_levels = num_levels;
  int prev = 0;
  const or_vt_node* node = vt_nodes;
  for (int i = 0; i < num_levels; ++i) {
    int ld = log_domain_sizes[i];
    if (ld < 0) {
      free(d);
      return set_err(OR_INVALID_ARGUMENT, "`log_domain_size` must be non-negative");
    }
    if (ld > 128) {
      free(d);
      return set_err(OR_INVALID_ARGUMENT, "`log_domain_size` must be <= 128");
    }
    if (i > 0 && ld <= prev) {
      free(d);
      return set_err(OR_INVALID_ARGUMENT,
                     "`log_domain_size` fields must be in ascending order in "
                     "`parameters`");
    }
    prev = ld;
    int st = vt_build(node, vt_node_counts[i], &d->vt[i]);
    node += vt_node_counts[i];
    if (st != OR_OK) {
      free(d);
      return st;
    }
    double sp = security_parameters[i];
    if (isnan(sp)) {
      free(d);
      return set_err(OR_INVALID_ARGUMENT, "`security_parameter` must not be NaN");
    }
    if (sp < 0 || sp > 128) {
      free(d);
      return set_err(OR_INVALID_ARGUMENT, "`security_parameter` must be in [0, 128]");
    }
    d->log_domain[i] = ld;
    /* Default security parameter (proto_validator.cc:43-46, 117-125). */
    d->security[i] = (sp == 0) ? 40.0 + ld : sp;
  }
  /* ProtoValidator::Create tree mapping (proto_validator.cc:127-153). */
  for (int t = 0; t < 130; ++t) d->tree_to_hierarchy[t] = -1;
  int tree_levels_needed = 0;
  for (int i = 0; i < num_levels; ++i) {
    int bits;
    int st = bits_needed_rec(d->vt[i].nodes, d->vt[i].num_nodes, d->security[i], &bits);
    if (st != OR_OK) {
      free(d);
      return st;
    }
    int log_bits_needed = (int)ceil(log2((double)bits));
    int tl = d->log_domain[i] - 7 + (log_bits_needed < 7 ? log_bits_needed : 7);
    if (tl < tree_levels_needed) tl = tree_levels_needed;
    d->tree_to_hierarchy[tl] = i;
    d->hierarchy_to_tree[i] = tl;
    tree_levels_needed = tree_levels_needed > tl + 1 ? tree_levels_needed : tl + 1;
    /* blocks_needed (cc:603-610). */
    d->blocks_needed[i] = (bits + 127) / 128;
  }
  d->tree_levels_needed = tree_levels_needed;
  prg_init(&d->prg_left, kPrgKeyLeft);
  prg_init(&d->prg_right, kPrgKeyRight);
  prg_init(&d->prg_value, kPrgKeyValue);
  *out = d;
  return OR_OK;
}

void or_dpf_free(or_dpf* dpf) { free(dpf); }
int or_dpf_tree_levels_needed(const or_dpf* d) { return d->tree_levels_needed; }
int or_dpf_hierarchy_to_tree(const or_dpf* d, int h) { return d->hierarchy_to_tree[h]; }
int or_dpf_blocks_needed(const or_dpf* d, int h) { return d->blocks_needed[h]; }
int or_dpf_num_scalars(const or_dpf* d, int h) { return d->vt[h].num_scalars; }
int or_dpf_elements_per_block(const or_dpf* d, int h) { return d->vt[h].epb; }
double or_dpf_security_parameter(const or_dpf* d, int h) { return d->security[h]; }

or_key* or_key_alloc(int num_cw, int num_levels, const int32_t* vc_count) {
  or_key* k = (or_key*)calloc(1, sizeof(or_key));
  if (!k) return NULL;
  k->num_cw = num_cw;
  k->num_levels = num_levels;
  k->cw_seed = (uint64_t*)calloc((size_t)(num_cw > 0 ? num_cw : 1) * 2, 8);
  k->cw_ccl = (uint8_t*)calloc((size_t)(num_cw > 0 ? num_cw : 1), 1);
  k->cw_ccr = (uint8_t*)calloc((size_t)(num_cw > 0 ? num_cw : 1), 1);
  k->vc_count = (int32_t*)calloc((size_t)num_levels, sizeof(int32_t));
  int total = 0;
  for (int i = 0; i < num_levels; ++i) {
    k->vc_count[i] = vc_count ? vc_count[i] : 0;
    total += k->vc_count[i];
  }
  k->vc = (uint64_t*)calloc((size_t)(total > 0 ? total : 1) * 2, 8);
  return k;
}

void or_key_free(or_key* k) {
  if (!k) return;
  free(k->cw_seed);
  free(k->cw_ccl);
  free(k->cw_ccr);
  free(k->vc_count);
  free(k->vc);
  free(k);
}

static const uint64_t* key_vc(const or_key* k, int h) {
  int off = 0;
  for (int i = 0; i < h; ++i) off += k->vc_count[i];
  return k->vc + 2 * off;
}

static int dpf_block_index_bits(const or_dpf* d, int h) {
  return d->log_domain[h] - d->hierarchy_to_tree[h];
}

/* DomainToTreeIndex / DomainToBlockIndex (cc:224-239). */
static u128 domain_to_tree_index(const or_dpf* d, u128 x, int h) {
  return x >> dpf_block_index_bits(d, h);
}
static int domain_to_block_index(const or_dpf* d, u128 x, int h) {
  int b = dpf_block_index_bits(d, h);
  return (int)(x & (((u128)1 << b) - 1));
}

static inline int extract_and_clear_lowest_bit(u128* x) {
  int bit = (int)(*x & 1);
  *x &= ~(u128)1;
  return bit;
}

/* ComputeValueCorrection (cc:81-117) + ComputeValueCorrectionFor<T>
 * (vth:614-648).  out: epb * ns words. */
static int compute_value_correction(const or_dpf* d, int h, const u128 seeds[2],
                                    u128 alpha, const u128* beta, int invert,
                                    u128* out) {
  int bn = d->blocks_needed[h];
  u128 exp[2 * 8];
  if (bn > 8) return set_err(OR_UNIMPLEMENTED, "blocks_needed too large");
  for (int j = 0; j < bn; ++j) {
    exp[j] = seeds[0] + (u128)j;
    exp[bn + j] = seeds[1] + (u128)j;
  }
  prg_evaluate(&d->prg_value, exp, exp, 2 * bn);
  int block_index = domain_to_block_index(d, alpha, h);
  const vtype_t* vt = &d->vt[h];
  int ns = vt->num_scalars, epb = vt->epb;
  u128 a[MAX_SCALARS * 16], b[MAX_SCALARS * 16];
  convert_bytes_to_array(vt, (const uint8_t*)exp, 16 * bn, a);
  convert_bytes_to_array(vt, (const uint8_t*)(exp + bn), 16 * bn, b);
  for (int s = 0; s < ns; ++s)
    b[block_index * ns + s] = s_add(&vt->scalars[s], b[block_index * ns + s], beta[s]);
  for (int e = 0; e < epb; ++e)
    for (int s = 0; s < ns; ++s) {
      const scalar_t* sc = &vt->scalars[s];
      u128 v = s_sub(sc, b[e * ns + s], a[e * ns + s]);
      if (invert) v = s_neg(sc, v);
      out[e * ns + s] = v;
    }
  return OR_OK;
}

/* ValidateValue (proto_validator.cc:289-333) for flattened scalars. */
static int validate_beta(const or_dpf* d, int h, const u128* beta) {
  const vtype_t* vt = &d->vt[h];
  for (int s = 0; s < vt->num_scalars; ++s) {
    const scalar_t* sc = &vt->scalars[s];
    if (sc->bits < 128 && beta[s] >= ((u128)1 << sc->bits)) {
      char v[64];
      u128_to_dec(beta[s], v);
      return set_err(OR_INVALID_ARGUMENT,
                     "Value (= %s) too large for ValueType with bitsize = %d", v,
                     sc->bits);
    }
    if (sc->kind == 3 && beta[s] >= sc->modulus) {
      char v[64], m[64];
      u128_to_dec(beta[s], v);
      u128_to_dec(sc->modulus, m);
      return set_err(OR_INVALID_ARGUMENT, "Value (= %s) is too large for modulus (= %s)", v, m);
    }
  }
  return OR_OK;
}

int or_generate_keys(const or_dpf* d, uint64_t alpha_lo, uint64_t alpha_hi,
                     const uint64_t* beta_words, const uint64_t seeds_in[4],
                     or_key** key0, or_key** key1) {
  u128 alpha = U128(alpha_lo, alpha_hi);
  int L = d->num_levels;
  u128 beta[130][MAX_SCALARS];
  int off = 0;
  for (int h = 0; h < L; ++h) {
    for (int s = 0; s < d->vt[h].num_scalars; ++s, ++off)
      beta[h][s] = load_u128(beta_words + 2 * off);
    int st = validate_beta(d, h, beta[h]);
    if (st != OR_OK) return st;
  }
  int last_ld = d->log_domain[L - 1];
  if (last_ld < 128 && alpha >= ((u128)1 << last_ld))
    return set_err(OR_INVALID_ARGUMENT, "`alpha` must be smaller than the output domain size");

  int32_t vc_count[130];
  for (int h = 0; h < L; ++h) vc_count[h] = d->vt[h].epb * d->vt[h].num_scalars;
  int ncw = d->tree_levels_needed - 1;
  or_key* k[2] = {or_key_alloc(ncw, L, vc_count), or_key_alloc(ncw, L, vc_count)};
  if (!k[0] || !k[1]) {
    or_key_free(k[0]);
    or_key_free(k[1]);
    return set_err(OR_RESOURCE_EXHAUSTED, "Memory allocation error");
  }
  k[0]->party = 0;
  k[1]->party = 1;
  u128 seeds[2] = {U128(seeds_in[0], seeds_in[1]), U128(seeds_in[2], seeds_in[3])};
  for (int p = 0; p < 2; ++p) store_u128(k[p]->seed, seeds[p]);
  int control_bits[2] = {0, 1};

  /* GenerateNext for tree levels 1..L-1 (cc:121-222). */
  for (int i = 1; i < d->tree_levels_needed; ++i) {
    int cw_idx = i - 1;
    if (d->tree_to_hierarchy[i - 1] >= 0) {
      int h = d->tree_to_hierarchy[i - 1];
      u128 alpha_prefix = 0;
      int shift = last_ld - d->log_domain[h];
      if (shift < 128) alpha_prefix = alpha >> shift;
      u128 vc[MAX_SCALARS * 16];
      int st = compute_value_correction(d, h, seeds, alpha_prefix, beta[h],
                                        control_bits[1], vc);
      if (st != OR_OK) {
        or_key_free(k[0]);
        or_key_free(k[1]);
        return st;
      }
      for (int p = 0; p < 2; ++p) {
        uint64_t* dst = (uint64_t*)key_vc(k[p], h);
        for (int j = 0; j < vc_count[h]; ++j) store_u128(dst + 2 * j, vc[j]);
      }
    }
    u128 e[2][2]; /* [branch][party] */
    prg_evaluate(&d->prg_left, seeds, e[0], 2);
    prg_evaluate(&d->prg_right, seeds, e[1], 2);
    int ecb[2][2];
    for (int b = 0; b < 2; ++b)
      for (int p = 0; p < 2; ++p) ecb[b][p] = extract_and_clear_lowest_bit(&e[b][p]);
    int current_bit = 0;
    if (last_ld - i < 128) current_bit = (int)((alpha >> (last_ld - i)) & 1);
    int keep = current_bit, lose = !current_bit;
    u128 seed_correction = e[lose][0] ^ e[lose][1];
    int cc[2];
    cc[0] = ecb[0][0] ^ ecb[0][1] ^ current_bit ^ 1;
    cc[1] = ecb[1][0] ^ ecb[1][1] ^ current_bit;
    for (int p = 0; p < 2; ++p) {
      seeds[p] = e[keep][p];
      if (control_bits[p]) seeds[p] ^= seed_correction;
    }
    for (int p = 0; p < 2; ++p)
      control_bits[p] = ecb[keep][p] ^ (control_bits[p] && cc[keep]);
    for (int p = 0; p < 2; ++p) {
      store_u128(k[p]->cw_seed + 2 * cw_idx, seed_correction);
      k[p]->cw_ccl[cw_idx] = (uint8_t)cc[0];
      k[p]->cw_ccr[cw_idx] = (uint8_t)cc[1];
    }
  }
  /* Last level value correction (cc:699-707). */
  u128 vc[MAX_SCALARS * 16];
  int st = compute_value_correction(d, L - 1, seeds, alpha, beta[L - 1],
                                    control_bits[1], vc);
  if (st != OR_OK) {
    or_key_free(k[0]);
    or_key_free(k[1]);
    return st;
  }
  for (int p = 0; p < 2; ++p) {
    uint64_t* dst = (uint64_t*)key_vc(k[p], L - 1);
    for (int j = 0; j < vc_count[L - 1]; ++j) store_u128(dst + 2 * j, vc[j]);
  }
  *key0 = k[0];
  *key1 = k[1];
  return OR_OK;
}

/* ProtoValidator::ValidateDpfKey (proto_validator.cc:205-236). */
static int validate_key(const or_dpf* d, const or_key* k) {
  if (k->num_levels != d->num_levels || k->vc_count[d->num_levels - 1] == 0)
    return set_err(OR_INVALID_ARGUMENT, "key.last_level_value_correction must be present");
  if (k->num_cw != d->tree_levels_needed - 1)
    return set_err(OR_INVALID_ARGUMENT,
                   "Malformed DpfKey: expected %d correction words, but got %d",
                   d->tree_levels_needed - 1, k->num_cw);
  for (int h = 0; h < d->num_levels; ++h) {
    if (d->hierarchy_to_tree[h] == d->tree_levels_needed - 1) continue;
    if (k->vc_count[h] == 0)
      return set_err(OR_INVALID_ARGUMENT,
                     "Malformed DpfKey: expected correction_words[%d] to contain "
                     "the value correction of hierarchy level %d",
                     d->hierarchy_to_tree[h], h);
  }
  return OR_OK;
}

/* ValuesToArray<T> (vth:561-580): size check. */
static int value_correction_array(const or_dpf* d, const or_key* k, int h,
                                  u128* out) {
  const vtype_t* vt = &d->vt[h];
  int want = vt->epb * vt->num_scalars;
  if (k->vc_count[h] != want)
    return set_err(OR_INVALID_ARGUMENT,
                   "values.size() (= %d) does not match ElementsPerBlock<T>() (= %d)",
                   vt->num_scalars ? k->vc_count[h] / vt->num_scalars : 0, vt->epb);
  const uint64_t* src = key_vc(k, h);
  for (int i = 0; i < want; ++i) out[i] = load_u128(src + 2 * i);
  return OR_OK;
}

/* --- EvaluateSeeds path walk (evaluate_prg_hwy.cc:552-634, 638-658) --- */
static int evaluate_seeds_impl(int64_t num_seeds, int num_levels,
                               int64_t num_cw, const u128* seeds_in,
                               const uint8_t* cb_in, const u128* paths,
                               int paths_rightshift, const u128* cw_seeds,
                               const uint8_t* ccl, const uint8_t* ccr,
                               const or_prg* prg_left, const or_prg* prg_right,
                               u128* seeds_out, uint8_t* cb_out) {
  if (num_cw != num_levels && num_cw != (int64_t)num_levels * num_seeds)
    return set_err(OR_INVALID_ARGUMENT,
                   "`num_correction_words` must be equal to `num_levels` or "
                   "`num_levels * num_seeds`");
  if (num_seeds == 0 || num_levels == 0) {
    if (num_levels == 0 && seeds_out != seeds_in) {
      for (int64_t i = 0; i < num_seeds; ++i) {
        seeds_out[i] = seeds_in[i];
        cb_out[i] = cb_in[i];
      }
    }
    return OR_OK;
  }
  /* Like the Highway path, evaluate one AES per seed and level using the
   * key selected by the path bit (identical result to NoHwy's two AES). */
  u128 buf[kBatchSize], out[kBatchSize];
  for (int64_t start = 0; start < num_seeds; start += kBatchSize) {
    int64_t bs = num_seeds - start < kBatchSize ? num_seeds - start : kBatchSize;
    for (int level = 0; level < num_levels; ++level) {
      const u128* s = (level == 0 ? seeds_in : seeds_out) + start;
      const uint8_t* cbp = (level == 0 ? cb_in : cb_out) + start;
      int bit_index = num_levels - level - 1 + paths_rightshift;
      int path_bits[kBatchSize];
      int cbs[kBatchSize];
      int nl = 0, nr = 0;
      int64_t li[kBatchSize], ri[kBatchSize];
      u128 lin[kBatchSize], rin[kBatchSize];
      for (int64_t i = 0; i < bs; ++i) {
        path_bits[i] = 0;
        if (bit_index < 128) path_bits[i] = (int)((paths[start + i] >> bit_index) & 1);
        cbs[i] = cbp[i];
        if (path_bits[i]) {
          ri[nr] = i;
          rin[nr++] = s[i];
        } else {
          li[nl] = i;
          lin[nl++] = s[i];
        }
      }
      prg_evaluate(prg_left, lin, buf, nl);
      for (int i = 0; i < nl; ++i) out[li[i]] = buf[i];
      prg_evaluate(prg_right, rin, buf, nr);
      for (int i = 0; i < nr; ++i) out[ri[i]] = buf[i];
      for (int64_t i = 0; i < bs; ++i) {
        int64_t ci = level;
        if (num_cw > num_levels) ci = (int64_t)level * num_seeds + start + i;
        u128 v = out[i];
        if (cbs[i]) v ^= cw_seeds[ci];
        int c = extract_and_clear_lowest_bit(&v);
        if (cbs[i]) c ^= path_bits[i] ? ccr[ci] : ccl[ci];
        seeds_out[start + i] = v;
        cb_out[start + i] = (uint8_t)c;
      }
    }
  }
  return OR_OK;
}

int or_evaluate_seeds(int64_t num_seeds, int num_levels,
                      int64_t num_correction_words, const uint64_t* seeds_in,
                      const uint8_t* control_bits_in, const uint64_t* paths,
                      int paths_rightshift, const uint64_t* correction_seeds,
                      const uint8_t* ccl, const uint8_t* ccr,
                      uint64_t key_left_lo, uint64_t key_left_hi,
                      uint64_t key_right_lo, uint64_t key_right_hi,
                      uint64_t* seeds_out, uint8_t* control_bits_out) {
  or_prg pl, pr;
  prg_init(&pl, U128(key_left_lo, key_left_hi));
  prg_init(&pr, U128(key_right_lo, key_right_hi));
  /* uint64 pairs have the u128 memory layout on x86-64 little endian. */
  return evaluate_seeds_impl(num_seeds, num_levels, num_correction_words,
                             (const u128*)seeds_in, control_bits_in,
                             (const u128*)paths, paths_rightshift,
                             (const u128*)correction_seeds, ccl, ccr, &pl, &pr,
                             (u128*)seeds_out, control_bits_out);
}

/* --- ExpandSeeds (cc:289-372) --- */
typedef struct {
  u128* seeds;
  uint8_t* cb;
  int64_t n;
} expansion_t;

static void expansion_free(expansion_t* e) {
  free(e->seeds);
  free(e->cb);
  e->seeds = NULL;
  e->cb = NULL;
}

static int expand_seeds(const or_dpf* d, const expansion_t* in,
                        const u128* cw_seeds, const uint8_t* ccl,
                        const uint8_t* ccr, int num_expansions,
                        expansion_t* out) {
  if (num_expansions >= 63)
    return set_err(OR_INVALID_ARGUMENT,
                   "Trying to expand more than 62 tree levels at once. Please "
                   "insert intermediate hierarchy levels, or evaluate fewer "
                   "hierarchy levels at once.");
  int64_t cur = in->n;
  int64_t out_size = cur << num_expansions;
  u128* a = (u128*)malloc(sizeof(u128) * (size_t)(out_size > 0 ? out_size : 1));
  u128* b = (u128*)malloc(sizeof(u128) * (size_t)(out_size > 0 ? out_size : 1));
  uint8_t* ca = (uint8_t*)malloc((size_t)(out_size > 0 ? out_size : 1));
  uint8_t* cbb = (uint8_t*)malloc((size_t)(out_size > 0 ? out_size : 1));
  if (!a || !b || !ca || !cbb) {
    free(a);
    free(b);
    free(ca);
    free(cbb);
    return set_err(OR_RESOURCE_EXHAUSTED, "Memory allocation error");
  }
  memcpy(a, in->seeds, sizeof(u128) * (size_t)cur);
  memcpy(ca, in->cb, (size_t)cur);
  u128 bl[kBatchSize], br[kBatchSize];
  for (int i = 0; i < num_expansions; ++i) {
    u128 cs = cw_seeds[i];
    int cl = ccl[i], cr = ccr[i];
    for (int64_t start = 0; start < cur; start += kBatchSize) {
      int64_t bs = cur - start < kBatchSize ? cur - start : kBatchSize;
      prg_evaluate(&d->prg_left, a + start, bl, bs);
      prg_evaluate(&d->prg_right, a + start, br, bs);
      for (int64_t j = 0; j < bs; ++j) {
        int64_t ie = 2 * (start + j);
        int t = ca[start + j];
        if (t) {
          bl[j] ^= cs;
          br[j] ^= cs;
        }
        b[ie] = bl[j];
        b[ie + 1] = br[j];
        cbb[ie] = (uint8_t)extract_and_clear_lowest_bit(&b[ie]);
        cbb[ie + 1] = (uint8_t)extract_and_clear_lowest_bit(&b[ie + 1]);
        if (t) {
          cbb[ie] ^= (uint8_t)cl;
          cbb[ie + 1] ^= (uint8_t)cr;
        }
      }
    }
    u128* ts = a;
    a = b;
    b = ts;
    uint8_t* tc = ca;
    ca = cbb;
    cbb = tc;
    cur *= 2;
  }
  free(b);
  free(cbb);
  out->seeds = a;
  out->cb = ca;
  out->n = cur;
  return OR_OK;
}

/* HashExpandedSeeds (cc:523-547). */
static u128* hash_expanded_seeds(const or_dpf* d, int h, const u128* seeds,
                                 int64_t n) {
  int bn = d->blocks_needed[h];
  u128* out = (u128*)malloc(sizeof(u128) * (size_t)(n * bn > 0 ? n * bn : 1));
  if (!out) return NULL;
  for (int64_t i = 0; i < n; ++i)
    for (int j = 0; j < bn; ++j) out[i * bn + j] = seeds[i] + (u128)j;
  prg_evaluate(&d->prg_value, out, out, n * bn);
  return out;
}

/* --- EvaluationContext ------------------------------------------------- */
struct or_ctx {
  const or_key* key;
  int previous_hierarchy_level;
  int partial_evaluations_level;
  int64_t num_pe;
  u128* pe_prefix;
  u128* pe_seed;
  uint8_t* pe_cb;
};

int or_ctx_create(const or_dpf* d, const or_key* key, or_ctx** out) {
  int st = validate_key(d, key);
  if (st != OR_OK) return st;
  or_ctx* c = (or_ctx*)calloc(1, sizeof(or_ctx));
  if (!c) return set_err(OR_RESOURCE_EXHAUSTED, "Memory allocation error");
  c->key = key;
  c->previous_hierarchy_level = -1;
  c->partial_evaluations_level = 0;
  *out = c;
  return OR_OK;
}

static void ctx_clear_pe(or_ctx* c) {
  free(c->pe_prefix);
  free(c->pe_seed);
  free(c->pe_cb);
  c->pe_prefix = c->pe_seed = NULL;
  c->pe_cb = NULL;
  c->num_pe = 0;
}

void or_ctx_free(or_ctx* c) {
  if (!c) return;
  ctx_clear_pe(c);
  free(c);
}
int or_ctx_previous_hierarchy_level(const or_ctx* c) { return c->previous_hierarchy_level; }
int or_ctx_partial_evaluations_level(const or_ctx* c) { return c->partial_evaluations_level; }
int64_t or_ctx_num_partial_evaluations(const or_ctx* c) { return c->num_pe; }
void or_ctx_partial_evaluations(const or_ctx* c, uint64_t* prefixes,
                                uint64_t* seeds, uint8_t* cbs) {
  for (int64_t i = 0; i < c->num_pe; ++i) {
    store_u128(prefixes + 2 * i, c->pe_prefix[i]);
    store_u128(seeds + 2 * i, c->pe_seed[i]);
    cbs[i] = c->pe_cb[i];
  }
}

typedef struct {
  u128 key;
  int64_t idx;
} kv_t;

static int cmp_kv(const void* a, const void* b) {
  u128 x = ((const kv_t*)a)->key, y = ((const kv_t*)b)->key;
  if (x < y) return -1;
  if (x > y) return 1;
  int64_t i = ((const kv_t*)a)->idx, j = ((const kv_t*)b)->idx;
  return (i > j) - (i < j);
}

/* ComputePartialEvaluations (cc:374-476). */
static int compute_partial_evaluations(const or_dpf* d, const u128* prefixes,
                                       int64_t n, int hierarchy_level,
                                       int update_ctx, or_ctx* ctx,
                                       expansion_t* out) {
  const or_key* key = ctx->key;
  int start_level = d->hierarchy_to_tree[ctx->partial_evaluations_level];
  int stop_level = d->hierarchy_to_tree[hierarchy_level];
  out->n = n;
  out->seeds = (u128*)malloc(sizeof(u128) * (size_t)(n > 0 ? n : 1));
  out->cb = (uint8_t*)malloc((size_t)(n > 0 ? n : 1));
  if (!out->seeds || !out->cb) {
    expansion_free(out);
    return set_err(OR_RESOURCE_EXHAUSTED, "Memory allocation error");
  }
  if (ctx->num_pe > 0 && start_level <= stop_level) {
    /* btree_map of previous partial evaluations (cc:388-406). */
    int64_t m = ctx->num_pe;
    kv_t* kv = (kv_t*)malloc(sizeof(kv_t) * (size_t)m);
    if (!kv) {
      expansion_free(out);
      return set_err(OR_RESOURCE_EXHAUSTED, "Memory allocation error");
    }
    for (int64_t i = 0; i < m; ++i) {
      kv[i].key = ctx->pe_prefix[i];
      kv[i].idx = i;
    }
    qsort(kv, (size_t)m, sizeof(kv_t), cmp_kv);
    /* First insertion wins; later duplicates must match (cc:399-405).  kv is
     * sorted by (key, idx), so the first entry of each group is the winner. */
    int64_t group_first = 0;
    for (int64_t i = 1; i < m; ++i) {
      if (kv[i].key != kv[i - 1].key) {
        group_first = i;
      } else {
        int64_t w = kv[group_first].idx, b = kv[i].idx;
        if (ctx->pe_seed[w] != ctx->pe_seed[b] || ctx->pe_cb[w] != ctx->pe_cb[b]) {
          free(kv);
          expansion_free(out);
          return set_err(OR_INVALID_ARGUMENT,
                         "Duplicate prefix in `ctx.partial_evaluations()` with "
                         "mismatching seed or control bit");
        }
      }
    }
    for (int64_t i = 0; i < n; ++i) {
      u128 pp = 0;
      if (stop_level - start_level < 128) pp = prefixes[i] >> (stop_level - start_level);
      int64_t lo = 0, hi = m;
      while (lo < hi) {
        int64_t mid = (lo + hi) / 2;
        if (kv[mid].key < pp)
          lo = mid + 1;
        else
          hi = mid;
      }
      if (lo >= m || kv[lo].key != pp) {
        free(kv);
        expansion_free(out);
        return set_err(OR_INVALID_ARGUMENT,
                       "Prefix not present in ctx.partial_evaluations at "
                       "hierarchy level %d",
                       hierarchy_level);
      }
      out->seeds[i] = ctx->pe_seed[kv[lo].idx];
      out->cb[i] = ctx->pe_cb[kv[lo].idx];
    }
    free(kv);
  } else {
    u128 seed = load_u128(key->seed);
    for (int64_t i = 0; i < n; ++i) {
      out->seeds[i] = seed;
      out->cb[i] = (uint8_t)key->party;
    }
    start_level = 0;
  }
  int nl = stop_level - start_level;
  u128* cws = (u128*)malloc(sizeof(u128) * (size_t)(nl > 0 ? nl : 1));
  for (int i = 0; i < nl; ++i) cws[i] = load_u128(key->cw_seed + 2 * (start_level + i));
  int st = evaluate_seeds_impl(n, nl, nl, out->seeds, out->cb, prefixes, 0, cws,
                               key->cw_ccl + start_level, key->cw_ccr + start_level,
                               &d->prg_left, &d->prg_right, out->seeds, out->cb);
  free(cws);
  if (st != OR_OK) {
    expansion_free(out);
    return st;
  }
  ctx_clear_pe(ctx);
  if (update_ctx && n > 0) {
    ctx->pe_prefix = (u128*)malloc(sizeof(u128) * (size_t)n);
    ctx->pe_seed = (u128*)malloc(sizeof(u128) * (size_t)n);
    ctx->pe_cb = (uint8_t*)malloc((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
      ctx->pe_prefix[i] = prefixes[i];
      ctx->pe_seed[i] = out->seeds[i];
      ctx->pe_cb[i] = out->cb[i];
    }
    ctx->num_pe = n;
  }
  ctx->partial_evaluations_level = hierarchy_level;
  return OR_OK;
}

/* ExpandAndUpdateContext (cc:478-521). */
static int expand_and_update_context(const or_dpf* d, int h, const u128* prefixes,
                                     int64_t n, or_ctx* ctx, expansion_t* out) {
  const or_key* key = ctx->key;
  expansion_t sel = {0};
  int start_level = 0;
  if (n == 0) {
    sel.n = 1;
    sel.seeds = (u128*)malloc(sizeof(u128));
    sel.cb = (uint8_t*)malloc(1);
    sel.seeds[0] = load_u128(key->seed);
    sel.cb[0] = (uint8_t)key->party;
  } else {
    int update_ctx = h < d->num_levels - 1;
    int st = compute_partial_evaluations(d, prefixes, n, ctx->previous_hierarchy_level,
                                         update_ctx, ctx, &sel);
    if (st != OR_OK) return st;
    start_level = d->hierarchy_to_tree[ctx->previous_hierarchy_level];
  }
  int stop_level = d->hierarchy_to_tree[h];
  int nl = stop_level - start_level;
  u128 cws[130];
  for (int i = 0; i < nl; ++i) cws[i] = load_u128(key->cw_seed + 2 * (start_level + i));
  int st = expand_seeds(d, &sel, cws, key->cw_ccl + start_level,
                        key->cw_ccr + start_level, nl, out);
  expansion_free(&sel);
  if (st != OR_OK) return st;
  ctx->previous_hierarchy_level = h;
  return OR_OK;
}

static void copy_out(const u128* src, int ns, uint64_t* dst) {
  for (int s = 0; s < ns; ++s) store_u128(dst + 2 * s, src[s]);
}

/* EvaluateUntil<T> (h:695-891). */
int or_evaluate_until(const or_dpf* d, int h, const uint64_t* prefix_words,
                      int64_t num_prefixes, or_ctx* ctx, uint64_t* out,
                      int64_t out_capacity, int64_t* out_count) {
  /* ValidateEvaluationContext (proto_validator.cc:238-267), parts that do
   * not concern proto parameter equality. */
  int st = validate_key(d, ctx->key);
  if (st != OR_OK) return st;
  if (ctx->previous_hierarchy_level >= d->num_levels - 1)
    return set_err(OR_INVALID_ARGUMENT, "This context has already been fully evaluated");
  if (ctx->num_pe > 0 && ctx->partial_evaluations_level > ctx->previous_hierarchy_level)
    return set_err(OR_INVALID_ARGUMENT,
                   "ctx.partial_evaluations_level must be less than or equal "
                   "to ctx.previous_hierarchy_level");
  if (h < 0 || h >= d->num_levels)
    return set_err(OR_INVALID_ARGUMENT,
                   "`hierarchy_level` must be non-negative and less than "
                   "parameters_.size()");
  if (h <= ctx->previous_hierarchy_level)
    return set_err(OR_INVALID_ARGUMENT,
                   "`hierarchy_level` must be greater than "
                   "`ctx.previous_hierarchy_level`");
  if ((ctx->previous_hierarchy_level < 0) != (num_prefixes == 0))
    return set_err(OR_INVALID_ARGUMENT,
                   "`prefixes` must be empty if and only if this is the first "
                   "call with `ctx`.");
  const u128* prefixes = (const u128*)prefix_words;
  int prev_ld = 0;
  int prev_h = ctx->previous_hierarchy_level;
  if (num_prefixes > 0) {
    prev_ld = d->log_domain[prev_h];
    for (int64_t i = 0; i < num_prefixes; ++i) {
      if (prev_ld < 128 && prefixes[i] >= ((u128)1 << prev_ld)) {
        char v[64];
        u128_to_dec(prefixes[i], v);
        return set_err(OR_INVALID_ARGUMENT,
                       "Index %s out of range for hierarchy level %d", v, prev_h);
      }
    }
  }
  int ld = d->log_domain[h];
  if (ld - prev_ld > 62)
    return set_err(OR_INVALID_ARGUMENT,
                   "Output size would be larger than 2**62. Please evaluate "
                   "fewer hierarchy levels at once.");
  const vtype_t* vt = &d->vt[h];
  int ns = vt->num_scalars;
  int cepb = 1 << (ld - d->hierarchy_to_tree[h]);
  int64_t opp = (int64_t)1 << (ld - prev_ld);
  int64_t total = num_prefixes > 0 ? num_prefixes * opp : opp;
  if (!out) {
    *out_count = total;
    return OR_OK;
  }
  if (out_capacity < total)
    return set_err(OR_INVALID_ARGUMENT, "output buffer too small");

  /* Tree index de-duplication (h:772-796). */
  u128* tree_indices = (u128*)malloc(sizeof(u128) * (size_t)(num_prefixes > 0 ? num_prefixes : 1));
  int64_t* pm_first = (int64_t*)malloc(sizeof(int64_t) * (size_t)(num_prefixes > 0 ? num_prefixes : 1));
  int* pm_second = (int*)malloc(sizeof(int) * (size_t)(num_prefixes > 0 ? num_prefixes : 1));
  int64_t num_tree = 0;
  if (num_prefixes > 0) {
    kv_t* kv = (kv_t*)malloc(sizeof(kv_t) * (size_t)num_prefixes);
    for (int64_t i = 0; i < num_prefixes; ++i) {
      kv[i].key = domain_to_tree_index(d, prefixes[i], prev_h);
      kv[i].idx = i;
    }
    qsort(kv, (size_t)num_prefixes, sizeof(kv_t), cmp_kv);
    /* first-appearance order: process prefixes in order, assign ids. */
    int64_t* first_of = (int64_t*)malloc(sizeof(int64_t) * (size_t)num_prefixes);
    for (int64_t i = 0; i < num_prefixes; ++i) {
      if (i > 0 && kv[i].key == kv[i - 1].key)
        first_of[kv[i].idx] = first_of[kv[i - 1].idx];
      else
        first_of[kv[i].idx] = kv[i].idx;
    }
    int64_t* id_of_first = (int64_t*)malloc(sizeof(int64_t) * (size_t)num_prefixes);
    for (int64_t i = 0; i < num_prefixes; ++i) {
      if (first_of[i] == i) {
        id_of_first[i] = num_tree;
        tree_indices[num_tree++] = domain_to_tree_index(d, prefixes[i], prev_h);
      }
      pm_first[i] = id_of_first[first_of[i]];
      pm_second[i] = domain_to_block_index(d, prefixes[i], prev_h);
    }
    free(kv);
    free(first_of);
    free(id_of_first);
  }
  expansion_t e = {0};
  st = expand_and_update_context(d, h, tree_indices, num_tree, ctx, &e);
  if (st != OR_OK) {
    free(tree_indices);
    free(pm_first);
    free(pm_second);
    return st;
  }
  int bn = d->blocks_needed[h];
  u128* hashed = hash_expanded_seeds(d, h, e.seeds, e.n);
  u128 corr[MAX_SCALARS * 16];
  st = value_correction_array(d, ctx->key, h, corr);
  if (st != OR_OK || !hashed) {
    free(hashed);
    expansion_free(&e);
    free(tree_indices);
    free(pm_first);
    free(pm_second);
    return st != OR_OK ? st : set_err(OR_RESOURCE_EXHAUSTED, "Memory allocation error");
  }
  int party = ctx->key->party;
  /* Per-leaf correction loop (h:836-862). */
  int64_t bptp = num_tree > 0 ? e.n / num_tree : e.n;
  u128 cur[MAX_SCALARS * 16];
  if (num_prefixes == 0) {
    for (int64_t i = 0; i < e.n; ++i) {
      convert_bytes_to_array(vt, (const uint8_t*)(hashed + i * bn), 16 * bn, cur);
      for (int j = 0; j < cepb; ++j) {
        for (int s = 0; s < ns; ++s) {
          u128 v = cur[j * ns + s];
          if (e.cb[i]) v = s_add(&vt->scalars[s], v, corr[j * ns + s]);
          if (party == 1) v = s_neg(&vt->scalars[s], v);
          cur[j * ns + s] = v;
        }
        copy_out(cur + j * ns, ns, out + 2 * ns * (i * cepb + j));
      }
    }
  } else {
    /* Gather per prefix (h:877-889). */
    for (int64_t p = 0; p < num_prefixes; ++p) {
      int64_t start = pm_first[p] * bptp * cepb + (int64_t)pm_second[p] * opp;
      for (int64_t k = 0; k < opp; ++k) {
        int64_t flat = start + k;
        int64_t i = flat / cepb;
        int j = (int)(flat % cepb);
        convert_bytes_to_array(vt, (const uint8_t*)(hashed + i * bn), 16 * bn, cur);
        for (int s = 0; s < ns; ++s) {
          u128 v = cur[j * ns + s];
          if (e.cb[i]) v = s_add(&vt->scalars[s], v, corr[j * ns + s]);
          if (party == 1) v = s_neg(&vt->scalars[s], v);
          cur[j * ns + s] = v;
        }
        copy_out(cur + j * ns, ns, out + 2 * ns * (p * opp + k));
      }
    }
  }
  *out_count = total;
  free(hashed);
  expansion_free(&e);
  free(tree_indices);
  free(pm_first);
  free(pm_second);
  return OR_OK;
}

/* EvaluateAtImpl<T> without context (h:913-1070). */
int or_evaluate_at(const or_dpf* d, const or_key* key, int h,
                   const uint64_t* point_words, int64_t n, uint64_t* out) {
  if (h < 0) return set_err(OR_INVALID_ARGUMENT, "`hierarchy_level` must be non-negative");
  if (h >= d->num_levels)
    return set_err(OR_INVALID_ARGUMENT,
                   "`hierarchy_level` must be less than the number of "
                   "parameters passed at construction");
  const u128* points = (const u128*)point_words;
  int ld = d->log_domain[h];
  u128 maxp = ~(u128)0;
  if (ld < 128) maxp = ((u128)1 << ld) - 1;
  for (int64_t i = 0; i < n; ++i)
    if (points[i] > maxp)
      return set_err(OR_INVALID_ARGUMENT,
                     "`evaluation_points[%lld]` larger than the domain size at "
                     "hierarchy level %d",
                     (long long)i, h);
  int st = validate_key(d, key);
  if (st != OR_OK) return st;
  if (n == 0) return OR_OK;
  const vtype_t* vt = &d->vt[h];
  int epb = vt->epb, ns = vt->num_scalars;
  u128* tree = (u128*)malloc(sizeof(u128) * (size_t)n);
  u128* seeds = (u128*)malloc(sizeof(u128) * (size_t)n);
  uint8_t* cb = (uint8_t*)malloc((size_t)n);
  for (int64_t i = 0; i < n; ++i) {
    tree[i] = epb > 1 ? domain_to_tree_index(d, points[i], h) : points[i];
    seeds[i] = load_u128(key->seed);
    cb[i] = (uint8_t)key->party;
  }
  int stop = d->hierarchy_to_tree[h];
  u128 cws[130];
  for (int i = 0; i < stop; ++i) cws[i] = load_u128(key->cw_seed + 2 * i);
  st = evaluate_seeds_impl(n, stop, stop, seeds, cb, tree, 0, cws, key->cw_ccl,
                           key->cw_ccr, &d->prg_left, &d->prg_right, seeds, cb);
  if (st != OR_OK) goto done;
  {
    int bn = d->blocks_needed[h];
    u128* hashed = hash_expanded_seeds(d, h, seeds, n);
    u128 corr[MAX_SCALARS * 16], cur[MAX_SCALARS * 16];
    st = value_correction_array(d, key, h, corr);
    if (st != OR_OK) {
      free(hashed);
      goto done;
    }
    for (int64_t i = 0; i < n; ++i) {
      convert_bytes_to_array(vt, (const uint8_t*)(hashed + i * bn), 16 * bn, cur);
      int bi = epb > 1 ? domain_to_block_index(d, points[i], h) : 0;
      for (int s = 0; s < ns; ++s) {
        u128 v = cur[bi * ns + s];
        if (cb[i]) v = s_add(&vt->scalars[s], v, corr[bi * ns + s]);
        if (key->party == 1) v = s_neg(&vt->scalars[s], v);
        store_u128(out + 2 * (i * ns + s), v);
      }
    }
    free(hashed);
  }
done:
  free(tree);
  free(seeds);
  free(cb);
  return st;
}

/* EvaluateAtImpl<T> with a context (h:356-378, 913-1070): the partial
 * evaluations stored in `ctx` are walked to `h`'s tree level by
 * ComputePartialEvaluations(tree_indices, h, update_ctx = true) (h:1000-1011),
 * so no further levels remain (start_level = stop_level), then the seeds are
 * hashed and corrected as without a context, and previous_hierarchy_level
 * becomes h (h:1065-1067). */
int or_evaluate_at_ctx(const or_dpf* d, int h, const uint64_t* point_words, int64_t n,
                       or_ctx* ctx, uint64_t* out) {
  if (h < 0) return set_err(OR_INVALID_ARGUMENT, "`hierarchy_level` must be non-negative");
  if (h >= d->num_levels)
    return set_err(OR_INVALID_ARGUMENT,
                   "`hierarchy_level` must be less than the number of "
                   "parameters passed at construction");
  const or_key* key = ctx->key;
  const u128* points = (const u128*)point_words;
  int ld = d->log_domain[h];
  u128 maxp = ~(u128)0;
  if (ld < 128) maxp = ((u128)1 << ld) - 1;
  for (int64_t i = 0; i < n; ++i)
    if (points[i] > maxp)
      return set_err(OR_INVALID_ARGUMENT,
                     "`evaluation_points[%lld]` larger than the domain size at "
                     "hierarchy level %d",
                     (long long)i, h);
  int st = validate_key(d, key);
  if (st != OR_OK) return st;
  if (n == 0) return OR_OK;
  const vtype_t* vt = &d->vt[h];
  int epb = vt->epb, ns = vt->num_scalars;
  u128* tree = (u128*)malloc(sizeof(u128) * (size_t)n);
  for (int64_t i = 0; i < n; ++i)
    tree[i] = epb > 1 ? domain_to_tree_index(d, points[i], h) : points[i];
  expansion_t sel = {0};
  st = compute_partial_evaluations(d, tree, n, h, 1, ctx, &sel);
  free(tree);
  if (st != OR_OK) return st;
  int bn = d->blocks_needed[h];
  u128* hashed = hash_expanded_seeds(d, h, sel.seeds, n);
  u128 corr[MAX_SCALARS * 16], cur[MAX_SCALARS * 16];
  st = value_correction_array(d, key, h, corr);
  if (st == OR_OK && hashed) {
    for (int64_t i = 0; i < n; ++i) {
      convert_bytes_to_array(vt, (const uint8_t*)(hashed + i * bn), 16 * bn, cur);
      int bi = epb > 1 ? domain_to_block_index(d, points[i], h) : 0;
      for (int s = 0; s < ns; ++s) {
        u128 v = cur[bi * ns + s];
        if (sel.cb[i]) v = s_add(&vt->scalars[s], v, corr[bi * ns + s]);
        if (key->party == 1) v = s_neg(&vt->scalars[s], v);
        store_u128(out + 2 * (i * ns + s), v);
      }
    }
    ctx->previous_hierarchy_level = h;
  } else if (st == OR_OK) {
    st = set_err(OR_RESOURCE_EXHAUSTED, "Memory allocation error");
  }
  free(hashed);
  expansion_free(&sel);
  return st;
}

/* Subtree slice of the last hierarchy level (CPU baseline workload). */
int or_expand_subtree(const or_dpf* d, const or_key* key, uint64_t first_lo,
                      uint64_t first_hi, int log_blocks, uint64_t* out) {
  int h = d->num_levels - 1;
  int L = d->hierarchy_to_tree[h];
  if (log_blocks > L || log_blocks > 40)
    return set_err(OR_INVALID_ARGUMENT, "log_blocks too large");
  u128 first = U128(first_lo, first_hi);
  int walk = L - log_blocks;
  u128 root_path = (walk < 128 && log_blocks < 128) ? (first >> log_blocks) : 0;
  u128 seed = load_u128(key->seed);
  uint8_t cb = (uint8_t)key->party;
  u128 cws[130];
  for (int i = 0; i < L; ++i) cws[i] = load_u128(key->cw_seed + 2 * i);
  int st = evaluate_seeds_impl(1, walk, walk, &seed, &cb, &root_path, 0, cws,
                               key->cw_ccl, key->cw_ccr, &d->prg_left,
                               &d->prg_right, &seed, &cb);
  if (st != OR_OK) return st;
  expansion_t root = {&seed, &cb, 1}, e = {0};
  st = expand_seeds(d, &root, cws + walk, key->cw_ccl + walk, key->cw_ccr + walk,
                    log_blocks, &e);
  if (st != OR_OK) return st;
  const vtype_t* vt = &d->vt[h];
  int ns = vt->num_scalars, bn = d->blocks_needed[h];
  int cepb = 1 << (d->log_domain[h] - L);
  u128* hashed = hash_expanded_seeds(d, h, e.seeds, e.n);
  u128 corr[MAX_SCALARS * 16], cur[MAX_SCALARS * 16];
  st = value_correction_array(d, key, h, corr);
  if (st == OR_OK && hashed) {
    for (int64_t i = 0; i < e.n; ++i) {
      convert_bytes_to_array(vt, (const uint8_t*)(hashed + i * bn), 16 * bn, cur);
      for (int j = 0; j < cepb; ++j)
        for (int s = 0; s < ns; ++s) {
          u128 v = cur[j * ns + s];
          if (e.cb[i]) v = s_add(&vt->scalars[s], v, corr[j * ns + s]);
          if (key->party == 1) v = s_neg(&vt->scalars[s], v);
          store_u128(out + 2 * ((i * cepb + j) * ns + s), v);
        }
    }
  }
  free(hashed);
  expansion_free(&e);
  return st;
}

/* ======================================================================== */
/* PIR inner product (inner_product_hwy.cc:45-74, 270-334)                   */
/* ======================================================================== */
int or_inner_product(int64_t num_values, const uint8_t* data,
                     const int64_t* offsets, const int64_t* sizes,
                     int num_queries, int64_t num_blocks,
                     const uint64_t* selections, int64_t max_value_size,
                     uint8_t* out) {
  if (num_queries == 0) return OR_OK;
  for (int i = 0; i < num_queries; ++i) {
    if (num_blocks * 128 < num_values)
      return set_err(OR_INVALID_ARGUMENT,
                     "`selections[%d]` contains insufficient number of bits: "
                     "%lld, expected: %lld",
                     i, (long long)(num_blocks * 128), (long long)num_values);
    if (max_value_size <= 0)
      return set_err(OR_INVALID_ARGUMENT, "`max_value_size` must be positive");
  }
  for (int64_t i = 0; i < num_values; ++i)
    if (sizes[i] > max_value_size)
      return set_err(OR_INVALID_ARGUMENT, "`values[%lld]` is larger than `max_value_size`",
                     (long long)i);
  memset(out, 0, (size_t)(num_queries * max_value_size));
  for (int64_t i = 0; i < num_blocks; ++i) {
    int64_t base = i * 128;
    for (int j = 0; j < 128; ++j) {
      if (base + j >= num_values) break;
      const uint8_t* v = data + offsets[base + j];
      int64_t sz = sizes[base + j];
      for (int k = 0; k < num_queries; ++k) {
        u128 sel = load_u128(selections + 2 * ((int64_t)k * num_blocks + i));
        if (((sel >> j) & 1) == 0) continue;
        uint8_t* r = out + (int64_t)k * max_value_size;
        for (int64_t b = 0; b < sz; ++b) r[b] ^= v[b];
      }
    }
  }
  return OR_OK;
}

/* AES-128-CTR keystream (AES_ctr128_encrypt with a zero nonce, big-endian
 * counter increment), aes_128_ctr_seeded_prng.cc:60-101. */
void or_aes_ctr_prng(const uint8_t seed[16], int64_t length, uint8_t* out) {
  uint8_t rk[176], ctr[16] = {0}, ks[16];
  aes128_expand_key(seed, rk);
  for (int64_t pos = 0; pos < length; pos += 16) {
    aes128_encrypt_blocks(rk, ctr, ks, 1);
    int64_t n = length - pos < 16 ? length - pos : 16;
    memcpy(out + pos, ks, (size_t)n);
    for (int i = 15; i >= 0; --i)
      if (++ctr[i] != 0) break;
  }
}
