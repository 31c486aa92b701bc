// host_aes.cc — see host_aes.h.  AES-NI when the CPU has it, otherwise the
// same T-table formulation the device uses.
#include "host_aes.h"

#include <string.h>
#include <sys/random.h>
#include <wmmintrin.h>
#include <smmintrin.h>

namespace dpf_amd {
namespace {

bool HaveAesNi() {
  static const bool have = __builtin_cpu_supports("aes");
  return have;
}

__attribute__((target("aes,sse4.1"))) void EncryptAesNi(const AesKey& k, const uint8_t* in,
                                                         uint8_t* out, size_t n) {
  __m128i rk[11];
  for (int r = 0; r < 11; ++r) rk[r] = _mm_loadu_si128(reinterpret_cast<const __m128i*>(&k.rk[4 * r]));
  size_t i = 0;
  for (; i + 4 <= n; i += 4) {
    __m128i b[4];
    for (int j = 0; j < 4; ++j)
      b[j] = _mm_xor_si128(_mm_loadu_si128(reinterpret_cast<const __m128i*>(in + 16 * (i + j))),
                           rk[0]);
    for (int r = 1; r < 10; ++r)
      for (int j = 0; j < 4; ++j) b[j] = _mm_aesenc_si128(b[j], rk[r]);
    for (int j = 0; j < 4; ++j)
      _mm_storeu_si128(reinterpret_cast<__m128i*>(out + 16 * (i + j)),
                       _mm_aesenclast_si128(b[j], rk[10]));
  }
  for (; i < n; ++i) {
    __m128i b = _mm_xor_si128(_mm_loadu_si128(reinterpret_cast<const __m128i*>(in + 16 * i)), rk[0]);
    for (int r = 1; r < 10; ++r) b = _mm_aesenc_si128(b, rk[r]);
    _mm_storeu_si128(reinterpret_cast<__m128i*>(out + 16 * i), _mm_aesenclast_si128(b, rk[10]));
  }
}

inline uint32_t Rotl(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }

void EncryptTable(const AesKey& k, const uint8_t* in, uint8_t* out, size_t n) {
  for (size_t i = 0; i < n; ++i) {
    uint32_t w[4];
    memcpy(w, in + 16 * i, 16);
    for (int c = 0; c < 4; ++c) w[c] ^= k.rk[c];
    for (int r = 1; r < 10; ++r) {
      uint32_t o[4];
      for (int c = 0; c < 4; ++c)
        o[c] = kTe0.t[w[c] & 0xff] ^ Rotl(kTe0.t[(w[(c + 1) & 3] >> 8) & 0xff], 8) ^
               Rotl(kTe0.t[(w[(c + 2) & 3] >> 16) & 0xff], 16) ^
               Rotl(kTe0.t[w[(c + 3) & 3] >> 24], 24) ^ k.rk[4 * r + c];
      memcpy(w, o, 16);
    }
    uint32_t o[4];
    for (int c = 0; c < 4; ++c)
      o[c] = (uint32_t)kSbox[w[c] & 0xff] | ((uint32_t)kSbox[(w[(c + 1) & 3] >> 8) & 0xff] << 8) |
             ((uint32_t)kSbox[(w[(c + 2) & 3] >> 16) & 0xff] << 16) |
             ((uint32_t)kSbox[w[(c + 3) & 3] >> 24] << 24);
    for (int c = 0; c < 4; ++c) o[c] ^= k.rk[40 + c];
    memcpy(out + 16 * i, o, 16);
  }
}

}  // namespace

HostAes::HostAes(u128 key)
    : key_(ExpandAesKey(static_cast<uint64_t>(key), static_cast<uint64_t>(key >> 64))) {}

HostAes::HostAes(const uint8_t kb[16]) {
  uint64_t lo, hi;
  memcpy(&lo, kb, 8);
  memcpy(&hi, kb + 8, 8);
  key_ = ExpandAesKey(lo, hi);
}

void HostAes::Encrypt(const uint8_t* in, uint8_t* out, size_t blocks) const {
  if (HaveAesNi())
    EncryptAesNi(key_, in, out, blocks);
  else
    EncryptTable(key_, in, out, blocks);
}

void HostAes::MmoHash(const u128* in, u128* out, size_t n) const {
  constexpr size_t kBatch = 64;
  u128 sigma[kBatch];
  for (size_t s = 0; s < n; s += kBatch) {
    size_t b = n - s < kBatch ? n - s : kBatch;
    for (size_t i = 0; i < b; ++i) {
      u128 x = in[s + i];
      uint64_t hi = static_cast<uint64_t>(x >> 64), lo = static_cast<uint64_t>(x);
      sigma[i] = (static_cast<u128>(hi ^ lo) << 64) | hi;
    }
    Encrypt(reinterpret_cast<const uint8_t*>(sigma), reinterpret_cast<uint8_t*>(out + s), b);
    for (size_t i = 0; i < b; ++i) out[s + i] ^= sigma[i];
  }
}

std::string AesCtrKeystream(const std::string& seed16, size_t offset, size_t length) {
  HostAes aes(reinterpret_cast<const uint8_t*>(seed16.data()));
  std::string out(length, '\0');
  size_t first_block = offset / 16;
  size_t end = offset + length;
  size_t nblocks = (end + 15) / 16 - first_block;
  std::string ctrs(16 * nblocks, '\0'), ks(16 * nblocks, '\0');
  for (size_t b = 0; b < nblocks; ++b) {
    // Big-endian 128-bit counter = first_block + b, starting from a zero IV.
    u128 c = static_cast<u128>(first_block + b);
    for (int j = 15; j >= 0; --j) {
      ctrs[16 * b + j] = static_cast<char>(c & 0xff);
      c >>= 8;
    }
  }
  aes.Encrypt(reinterpret_cast<const uint8_t*>(ctrs.data()),
              reinterpret_cast<uint8_t*>(&ks[0]), nblocks);
  memcpy(&out[0], ks.data() + (offset - 16 * first_block), length);
  return out;
}

bool SecureRandom(void* buf, size_t len) {
  uint8_t* p = static_cast<uint8_t*>(buf);
  while (len > 0) {
    ssize_t r = getrandom(p, len, 0);
    if (r <= 0) return false;
    p += r;
    len -= static_cast<size_t>(r);
  }
  return true;
}

}  // namespace dpf_amd
