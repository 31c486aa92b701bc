// host_aes.h — host AES-128 for the host-only parts of the protocol: key
// generation (GenerateKeysIncremental, cc:642-710 — a client-side operation
// the reference also runs on the CPU) and the Helper's AES-CTR one-time pad
// (pir/prng/aes_128_ctr_seeded_prng.cc).  DPF *evaluation* never uses this
// code: it runs in the gfx950 kernels.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <string>

#include "aes_tables.h"

namespace dpf_amd {

class HostAes {
 public:
  explicit HostAes(u128 key);
  HostAes(const uint8_t key_bytes[16]);  // NOLINT
  // out[i] = AES_k(in[i]) on 16-byte blocks.
  void Encrypt(const uint8_t* in, uint8_t* out, size_t blocks) const;
  // Aes128FixedKeyHash::Evaluate (aes_128_fixed_key_hash.cc:57-98).
  void MmoHash(const u128* in, u128* out, size_t n) const;

 private:
  AesKey key_;
};

// Aes128CtrSeededPrng::GetRandomBytes stream (zero nonce, big-endian
// counter): bytes [offset, offset + length) of the key stream.
std::string AesCtrKeystream(const std::string& seed16, size_t offset, size_t length);

// Cryptographically secure random bytes (getrandom(2)); replaces RAND_bytes.
bool SecureRandom(void* buf, size_t len);

}  // namespace dpf_amd
